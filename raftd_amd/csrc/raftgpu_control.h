// raftgpu_control.h — the per-replica Raft step (control_kernel<R>'s body), kept in a header so
// the same code compiles for the GPU (RG_FN = __device__ __forceinline__) and, in the test-only
// host harness tests/native/ctl_host.cpp, for the CPU under AddressSanitizer.
// Semantics: DESIGN.md §1 (dragonboat v4 internal/raft restated).
#pragma once
#include "raftgpu_internal.h"

#include <type_traits>

// Fast paths of the control step (on; RG_CTL_SLOW turns all three off for A/B runs):
//   RG_CTL_FASTREP   a leader builds the Replicate of its own same-step append from registers and
//                    sends it as a uniform Replicate (one inline word for all n entries, below)
//   RG_CTL_FRESH     write_entries' fresh-index path (pointer-stepped ring slots, no hull)
//   RG_CTL_HDRBATCH  handle() loads all eight header words of a message up front
//   RG_CTL_LTCACHE   term_at keeps the term of one index (at first `last`) in registers
// Uniform Replicate: header word 7 = RG_UNIFORM marks a local Replicate whose n entries all carry
// the ring word mt[0] (only mt[0] is written). Remote Replicates never carry it: unpack_kernel
// replaces word 7 with the records' offset, and pack_kernel expands the word into n records.
#ifndef RG_CTL_SLOW
#ifndef RG_CTL_FASTREP
#define RG_CTL_FASTREP
#endif
#ifndef RG_CTL_FRESH
#define RG_CTL_FRESH
#endif
#ifndef RG_CTL_HDRBATCH
#define RG_CTL_HDRBATCH
#endif
#ifndef RG_CTL_LTCACHE
#define RG_CTL_LTCACHE
#endif
#endif

// entries per load batch in the control kernel's term copies (write_entries, send_replicate)
#ifndef RG_CTL_FULL_BATCH
#define RG_CTL_FULL_BATCH 2
#endif
#ifndef RG_CTL_BATCH
#define RG_CTL_BATCH 8
#endif

// RG_CTL_PROFILE (measurement builds): shader-clock stamps at the phase boundaries of a step
#if defined(RG_CTL_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
#define RG_STAMP(i) (stamps[i] = (uint32_t)__builtin_amdgcn_s_memtime())
// accumulated time of a sub-phase (acc[i] += cycles since t0), rows 6.. of the profile
#define RG_T0(v) const uint32_t v = (uint32_t)__builtin_amdgcn_s_memtime()
#define RG_ACC(i, t0) (stamps[6 + (i)] += (uint32_t)__builtin_amdgcn_s_memtime() - (t0))
#else
#define RG_STAMP(i) ((void)0)
#define RG_T0(v) ((void)0)
#define RG_ACC(i, t0) ((void)0)
#endif

#ifndef RG_FN
#define RG_FN __device__ __forceinline__
#endif

namespace rg {
#ifdef RG_X1
#define RGX(c) true
#else
#define RGX(c) (c)
#endif
#ifdef RG_X2
#define RGX2(c) true
#else
#define RGX2(c) (c)
#endif

RG_FN uint64_t mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ULL;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return z;
}
RG_FN uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }
RG_FN uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }

// ================================================================== control kernel
// Compile-time loop: f(integral_constant<int, J>) for J = B .. E-1, fully unrolled.
template <int B, int E, class F>
RG_FN void sfor(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sfor<B + 1, E>(f);
  }
}
// remote slot f of a per-replica array, with constant indices only (the arrays stay in registers)
// Diagnostic variants (RG_AB_SV_*): Ctl's slot in one class of uses is laundered through a VGPR
// move (Ctl::slot_lane), so the compiler treats it as per-lane there (the fault)
#ifndef RG_CTL_RELOAD_FAST
#define RG_CTL_RELOAD_FAST 0
#endif
// the large-engine fast step (LEAN) reloads the parameter fields too: with the state updated in place
// its hoisted pointers pushed control_fast_kernel<3> past 168 VGPRs (58 spilled to scratch); reloaded,
// 145 VGPRs and no scratch. r05's A/B had it neutral at 64K x 3 and C5 (r05l); the LAT build of small
// engines keeps the hoisted loads (reloading cost C2 ~5 µs there)
#ifndef RG_CTL_RELOAD_LEAN
#define RG_CTL_RELOAD_LEAN 1
#endif
#ifdef RG_AB_SV_SEND
#define RG_S_SEND slot_lane()
#else
#define RG_S_SEND s
#endif
#ifdef RG_AB_SV_INBOX
#define RG_S_INBOX slot_lane()
#else
#define RG_S_INBOX s
#endif
#ifdef RG_AB_SV_ID
#define RG_S_ID slot_lane()
#else
#define RG_S_ID s
#endif

template <int R, class T>
RG_FN T sel_get(const T (&a)[R], uint32_t f) {
  T v = a[0];
  sfor<1, R>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    v = (uint32_t)j == f ? a[j] : v;
  });
  return v;
}
template <int R, class T, class V>
RG_FN void sel_set(T (&a)[R], uint32_t f, V val) {
  sfor<0, R>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    a[j] = (uint32_t)j == f ? (T)val : a[j];
  });
}

// The parameter block is read through the constant address space on the device: it does not
// change during a launch, so every field read is a scalar (s_load) read served by the scalar cache,
// wherever it sits in the step (stores to global memory cannot clobber it), and no copy of the
// block has to stay live in registers.
#if defined(__HIP_DEVICE_COMPILE__)
#define RG_CONST(T) __attribute__((address_space(4))) T
#else
#define RG_CONST(T) T
#endif
using CTickParams = RG_CONST(const TickParams);

// FAST = true: the steady-state step (control_fast_kernel, DESIGN.md §3 "Fast path"). It implements the
// paths a replica takes in steady state — a leader handling ReplicateResp / HeartbeatResp, ticking,
// appending its synthetic proposal batch and replicating it; a follower appending a uniform Replicate at
// its log end, committing and answering heartbeats — and ABORTS at every other branch (elections, term
// changes, rejections, truncation, snapshots, membership changes, reads, caller Cmds, remote messages).
// An aborted lane stores nothing: the full kernel (FAST = false) re-runs its whole step from the same
// inputs. Every memory write the fast path made before aborting is one the full step makes too (same
// decisions on the same inputs: outbox slots, fresh ring words past the old log end, job rows, S_NLPG),
// or lies where nothing reads it (message slots past the final count, ring slots past the final last,
// job rows past the final job count). Fewer live values: the fields only the aborted branches touch are
// copied through at the end instead of living in registers for the whole step.
// ROLE (FAST only): -1 = any role; LEADER / FOLLOWER = the role-sorted fast launches (control_fast_kernel):
// the lane's role is that compile-time constant for the whole step (the fast path never changes a role:
// every transition aborts), so the other roles' branches compile away.
// LAT (FAST only): the latency build for small engines (control_fastfb_kernel, the resident kernel:
// a wave or less per SIMD, registers to spare) loads every field with the state up front instead of
// copying the cold ones through at the end (one round trip fewer on the step's critical path).
// SLIM (full step only): load batches of RG_CTL_FULL_BATCH entries instead of RG_CTL_BATCH — the
// build of control_slow_kernel / control_kernel, whose live values then fit the register file (no
// VGPR spills at R <= 5); the fallback inside control_fastfb_kernel keeps the wide batches (r05ac: the
// narrow ones cost C2's fused launch ~2 µs, the storm's slow kernel nothing)
template <int R, bool FAST = false, int ROLE = -1, bool LAT = false, bool SLIM = false>
struct Ctl {
  // LEAN: the fields only the end of the step reads (processed, applied, snapshot index, cc_hi) are
  // loaded there, not with the state (register-lean); LAT loads them up front
  static constexpr bool LEAN = FAST && !LAT;
  // the tick's parameter block, read in place at each use (a device slot the host filled): the
  // fields are reloaded where needed instead of living in registers for the whole step (r02 kept a
  // 368-B copy, 279 SGPR spills at R = 3)
  CTickParams& p_;
  // P(): the parameter block. In the full step (FAST = false; the fast step too with
  // RG_CTL_RELOAD_FAST) each use loads the field it needs through a pointer the compiler cannot see
  // through, so the loads are not hoisted to the kernel entry and no pointer stays live in an SGPR
  // for the whole step: control_slow_kernel<3> 456 → 66 SGPR spills (into VGPR lanes), <5> 429 → 72.
  // A field is one scalar-cache hit away at each use. RG_AB_CTL_HOIST: r04's hoisted loads (A/B)
  RG_FN CTickParams& P() const {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(RG_AB_CTL_HOIST)
    if constexpr (!FAST || RG_CTL_RELOAD_FAST || (LEAN && RG_CTL_RELOAD_LEAN)) {
      CTickParams* r = &p_;
      asm volatile("" : "+s"(r));
      return *r;
    }
#endif
    return p_;
  }
  bool aborted = false;  // FAST: the step left the fast path (the full kernel re-runs it)
  uint32_t q, g, s;    // g = local column (indexes every device array)
  uint64_t gg, rid;    // global group and global replica id gg·R + s (RNG keys, loss hash)
  uint32_t gi;         // the global group as an index into this engine's tick-input arrays (< 2^32)
  uint64_t term, vote, leader, committed, applied, last, marker, marker_term, snap_index, snap_term, cap_base;
  uint64_t processed;  // committed entries handed to the state machine (entryLog.processed)
  uint32_t role, etick, htick, rand_to, rng_ctr, granted, responded, active, err, drops;
  uint32_t members, snap_members, cc_pending;  // membership
  uint64_t cc_hi;                              // highest index a ConfigChange entry was written to
  // remote match / next / snapshot index; at R = 8 the snapshot indices (touched only on the
  // snapshot path) stay in this step's output rows instead of registers
  static constexpr bool RS_MEM = R >= 8;
  // The fast step neither reads nor writes the snapshot indices: a remote's rsnap is non-zero only in
  // the SNAPSHOT state, and every SNAPSHOT branch leaves the fast path (rs_get / rs_set below)
  static constexpr bool RS_REG = !RS_MEM && !FAST;
  uint64_t rm[R], rn[R], rs[RS_REG ? R : 1];
  uint32_t rt[R];                // remote state
  uint64_t last_start, sent_hi, rw_lo, rw_hi, marker_start;
  uint64_t processed_start, restored_at;  // apply window: entries restored from a snapshot are not Update()d
  bool took;                            // a snapshot was taken at the end of this step
  uint64_t wlo;                         // lowest log index written this step (EntriesToSave from here)
  // payload stream: hw = next free chunk. The lowest page held (S_LPG, the capacity
  // rule's base, unchanged during a step) is read where an append needs it
  uint32_t hw;
  uint32_t lpg_;   // S_LPG at step start (read with the state; the capacity rule's base)
  uint32_t nlpg_;  // S_NLPG out: pages below it are released after this step (pool_kernel)
  // RG_CTL_FASTREP (see the top of this file). The leader's last append
  // of this step when it wrote no protected index: entries
  // [la_base, la_base + la_n) all hold the ring word la_word (bank 0) and term(la_base − 1) = la_pt,
  // their Cmds start at stream chunk la_pos, so send_replicate builds a Replicate of them from
  // registers instead of re-reading the ring. la_n = 0 when any other log write, reset or restore
  // came after it.
#ifdef RG_CTL_FASTREP
  uint64_t la_base, la_word, la_pt;
  uint32_t la_n, la_pos;
#endif
  uint64_t oc, em;  // per destination: enqueued / emitted counts, 8 bits each
  uint64_t ocls;    // per destination: the classes of its first four messages (2 bits each, cnt_cls)
  uint32_t nj;      // jobs emitted
  uint64_t lt_i = ~0ull, lt_v = 0;  // term_at cache: index lt_i has term lt_v (~0: none)
  // in-place store (FAST): what the step changed, for the fields it cannot compare at the end
  uint32_t etick0 = 0, drops0 = 0;  // at step start
  bool ldv = false, cmv = false;    // leader / committed moved

  RG_FN Ctl(CTickParams& pp, uint32_t qq) : Ctl(pp, qq / pp.G, qq - (qq / pp.G) * pp.G) {}
  // slot ss of group column g0: the kernels pass a wave-uniform slot (the grid's y index), so every
  // value derived from s alone (its outbox planes, the sender loop's skip, my_id) stays scalar
  RG_FN Ctl(CTickParams& pp, uint32_t ss, uint32_t g0) : p_(pp), q(ss * pp.G + g0), g(g0), s(ss) {
    gg = pl_group(P().pl, RG_S_ID, g);
    rid = gg * R + RG_S_ID;
    gi = (uint32_t)pl_input_index(P().pl, gg);
    const uint64_t n = P().nrep;
    const uint64_t* a = P().s64 + q;
    const uint32_t* b = P().s32 + q;
    term = a[S_TERM * n]; leader = a[S_LEADER * n]; committed = a[S_COMMITTED * n];
    last = a[S_LAST * n]; marker = a[S_MARKER * n]; marker_term = a[S_MARKER_TERM * n];
    cap_base = a[S_CAP_BASE * n];
    role = b[S_ROLE * n]; etick = b[S_ETICK * n]; htick = b[S_HTICK * n]; rand_to = b[S_RAND_TO * n];
    active = b[S_ACTIVE * n]; drops = b[S_DROPS * n]; members = b[S_MEMBERS * n];
    hw = b[S_HW * n];
    if constexpr (!FAST) {  // the fields no fast branch reads or changes (it aborts first): not loaded there
      vote = a[S_VOTE * n]; snap_term = a[S_SNAP_TERM * n];
      rng_ctr = b[S_RNG_CTR * n]; granted = b[S_GRANTED * n]; responded = b[S_RESPONDED * n];
      err = b[S_ERR * n]; snap_members = b[S_SNAP_MEMBERS * n]; cc_pending = b[S_CC_PENDING * n];
    } else {
      vote = snap_term = 0;
      rng_ctr = granted = responded = err = snap_members = cc_pending = 0;
    }
    if constexpr (!LEAN) {
      applied = a[S_APPLIED * n]; snap_index = a[S_SNAP_INDEX * n]; processed = a[S_PROCESSED * n];
      cc_hi = a[S_CC_HI * n];
    } else {
      applied = snap_index = processed = cc_hi = 0;
    }
    etick0 = etick;
    drops0 = drops;
    sfor<0, R>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      rm[j] = P().rem[(0 * R + j) * n + q];
      rn[j] = P().rem[(1 * R + j) * n + q];
      if constexpr (RS_REG) rs[j] = P().rem[(2 * R + j) * n + q];
      else rs[0] = 0;  // RS_MEM: read and written in place (rs_get / rs_set); FAST: never touched
      rt[j] = P().rst[j * n + q];
    });
#ifdef RG_AB_LAST_TERM_RING  // A/B variant: the term of `last` from the ring (r04)
    if (last > marker) lt_set(last, *tr_at(last) & TERM_MASK);
#else
    if (last > marker) lt_set(last, a[S_LAST_TERM * n]);  // the state row: no ring read
#endif
    last_start = last; sent_hi = 0; rw_lo = ~0ull; rw_hi = 0; marker_start = marker;
    processed_start = processed; restored_at = 0; wlo = ~0ull; took = false;
    if constexpr (FAST) {
      if (role == CANDIDATE) abort_();  // every candidate path (votes, fallback) is the full step's
      if constexpr (ROLE >= 0) role = ROLE;  // the launch's role (the kernel stepped only those lanes)
    }
    // the last step compacted (or restored) to the marker (it moved off cap_base, the marker that
    // step started from; rg_compact moves it the same way between ticks): entry marker + 1's stream
    // position bounds the pages to release, known now that the step which wrote it has stored its
    // {crc, position} (the bulk kernel). They go back to the pool at the end of this step; the capacity rule keeps lpg until
    // then, so a page read in this launch is never reassigned in it
    lpg_ = b[S_LPG * n];
    {
      uint32_t nlpg = lpg_;
      if (marker != cap_base) {
        const uint64_t fi = marker + 1;
        uint32_t bound = hw;
        if (fi <= last) {
          const uint64_t sl = fi & (P().L - 1), bank = *tr_at(fi) >> 63;
          bound = P().info[(bank * n + q) * P().L + sl].y;
        }
        nlpg = vpn_of(bound);
      }
      nlpg_ = nlpg;  // for pool_kernel, stored with the state (no store before the inbox: the step's
                     // loads up to its first message can all be in flight together)
    }
#ifdef RG_CTL_FASTREP
    la_base = la_word = la_pt = 0; la_n = 0; la_pos = 0;
#endif
    oc = 0; em = 0; ocls = 0; nj = 0;
  }

  // entries per load batch (RG_CTL_BATCH); at R >= 7 the remote arrays leave room for half as many
  static constexpr uint32_t CB = SLIM ? RG_CTL_FULL_BATCH
                                      : R >= 7 ? (RG_CTL_BATCH > 4 ? 4 : RG_CTL_BATCH) : RG_CTL_BATCH;
  RG_FN uint64_t ri() const { return (uint64_t)gi * R + RG_S_ID; }  // the replica's tick-input index
  RG_FN void abort_() { aborted = true; }  // FAST: leave the fast path (the full kernel re-runs the step)
  RG_FN uint32_t quorum() const { return (uint32_t)__builtin_popcount(members) / 2 + 1; }  // voting members
  RG_FN bool is_member(uint32_t i) const { return (members >> i) & 1u; }
  // Diagnostic variants (RG_AB_SV_*; DESIGN.md §3, the control-kernel fault): the slot, laundered
  // through a VGPR move so the compiler treats it as per-lane, in one class of uses at a time
  RG_FN uint32_t slot_lane() const {
    uint32_t v = s;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("v_mov_b32 %0, %0" : "+v"(v));
#endif
    return v;
  }
  RG_FN uint32_t my_id() const { return RG_S_ID + 1; }

  // ---- remotes (compile-time R: selects, no local-memory arrays)
#define RG_GET(arr, f) sel_get<R>(arr, f)
#define RG_SET(arr, f, val) sel_set<R>(arr, f, val)
  // FAST: 0 and a no-op. The fast step reaches them only where a remote leaves RETRY for REPLICATE
  // (respondedTo), whose rsnap is already 0; an aborted fast step must not have written state in place
  RG_FN uint64_t rs_get(uint32_t f) const {
    if constexpr (FAST) return 0;
    else if constexpr (RS_MEM) return P().rem[((uint64_t)(2 * R) + f) * P().nrep + q];
    else return sel_get<R>(rs, f);
  }
  RG_FN void rs_set(uint32_t f, uint64_t v) {
    if constexpr (FAST) {
      (void)f; (void)v;
    } else if constexpr (RS_MEM) {
      P().rem[((uint64_t)(2 * R) + f) * P().nrep + q] = v;
    } else {
      sel_set<R>(rs, f, v);
    }
  }

  // ---- log (entryLog)
  RG_FN uint64_t* tr_at(uint64_t i) const {
    return P().tr + (uint64_t)(i & (P().L - 1)) * P().nrep + q;
  }
  RG_FN uint64_t term_at(uint64_t i) const {
    if (i == marker) return marker_term;
    if (i > marker && i <= last) return i == lt_i ? lt_v : *tr_at(i) & TERM_MASK;
    return 0;
  }
  // the term of one index kept in registers (RG_CTL_LTCACHE): the step's own writes keep it
  // current (write_entries_), so the repeated term_at(last) of a leader's commit checks and
  // empty Replicates and a follower's log-matching check cost no ring round trip
  RG_FN void lt_set(uint64_t i, uint64_t t) {
#ifdef RG_CTL_LTCACHE
    if constexpr (R < 8) {  // at R = 8 the two registers push the lane into scratch: off there
      lt_i = i;
      lt_v = t;
    }
#else
    (void)i;
    (void)t;
#endif
  }
  RG_FN void commit_to(uint64_t i) {
    if (i <= committed) return;
    if (i > last) {
      if constexpr (FAST) {
        abort_();
        return;
      }
      err |= ERR_BEYOND;
      return;
    }
    committed = i;
    cmv = true;
  }

  // ---- transport
  RG_FN static uint32_t get8(uint64_t packed, uint32_t d) {
    return (uint32_t)(packed >> (8 * d)) & 0xFF;
  }
  RG_FN bool lost(uint32_t dst, uint32_t n) const {
    if (P().isolate && (P().isolate[ri()] || P().isolate[(uint64_t)gi * R + dst])) return true;
    if (P().drop_ppm) {
      uint64_t h = mix64(P().seed ^ mix64((P().tick << 40) ^ ((uint64_t)rid << 8) ^ dst) ^ (uint64_t)(n + 1));
      if (h % 1000000ull < P().drop_ppm) return true;
    }
    return false;
  }
  // raft.send + enqueue into the outbox slot (SoA). Returns slot k, or -1 if lost.
  RG_FN int send(uint32_t type, uint32_t to, uint64_t mterm, uint32_t reject, uint32_t nent,
                                      uint64_t log_term, uint64_t log_index, uint64_t commit, uint64_t hint,
                                      uint64_t hint_high, uint32_t src_a, uint32_t src_b) {
    const uint32_t dst = to - 1;
    if (dst >= (uint32_t)R) {  // unreachable with validated inputs (handle() and unpack check ids)
      if constexpr (FAST) {
        abort_();
        return -1;
      }
      err |= ERR_WIRE;
      return -1;
    }
    if (type != M_PROPOSE && type != M_REQUEST_VOTE && type != M_READ_INDEX) mterm = term;
    const uint32_t n = get8(em, dst);
    em += 1ull << (8 * dst);
    const uint32_t k = get8(oc, dst);
    if (lost(dst, n) || k >= P().K) {
      drops++;
      return -1;
    }
    oc += 1ull << (8 * dst);
    // the fast step classifies its messages for the receivers; the full step's (rare: elections,
    // recoveries) stay MC_ALL, which a receiver always reads correctly (every word)
    if constexpr (FAST) {
      if (k < 4) ocls |= (uint64_t)msg_class(type, nent) << (8 * dst + 2 * k);
    }
    const uint64_t plane = (uint64_t)R * R * P().K * P().G;
    uint64_t* h = P().hdr_out + (((uint64_t)RG_S_SEND * R + dst) * P().K + k) * P().G + g;
    const uint32_t wm = hdr_words(type, nent);  // the words this message carries (per type, and an empty Replicate's)
    h[0 * plane] = (uint64_t)type | ((uint64_t)my_id() << 8) | ((uint64_t)to << 16) | ((uint64_t)reject << 24) |
                   ((uint64_t)nent << 32);
    h[1 * plane] = mterm;
    if (wm & 0x04u) h[2 * plane] = log_term;
    if (wm & 0x08u) h[3 * plane] = log_index;
    if (wm & 0x10u) h[4 * plane] = commit;
    if (wm & 0x20u) h[5 * plane] = hint;
    if (wm & 0x40u) h[6 * plane] = hint_high;
    if (wm & 0x80u) h[7 * plane] = (uint64_t)src_a | ((uint64_t)src_b << 32);
    return (int)k;
  }
  RG_FN int send_simple(uint32_t type, uint32_t to, uint32_t reject = 0, uint64_t log_index = 0,
                                             uint64_t hint = 0, uint64_t hint_high = 0) {
    return send(type, to, 0, reject, 0, 0, log_index, 0, hint, hint_high, 0, 0);
  }

  // ---- role transitions (A.5)
  RG_FN void reset(uint64_t t) {
    if (t != term) {
      term = t;
      vote = 0;
    }
    leader = 0;
    granted = responded = 0;
    etick = htick = 0;
    rng_ctr++;
    uint64_t key = (gg << 32) | ((uint64_t)s << 24) | (uint64_t)(rng_ctr & 0xFFFFFF);
    rand_to = P().ET + (uint32_t)(mix64(P().seed ^ mix64(key)) % P().ET);
    sfor<0, R>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      rm[j] = (uint32_t)j == s ? last : 0;
      rn[j] = last + 1;
      rs_set(j, 0);
      rt[j] = RETRY;
    });
    active = 0;
    cc_pending = 0;  // clearPendingConfigChange
    if (P().rdst) P().rdst[(uint64_t)RQ_N * P().nrep + q] = 0;  // readIndex.reset: a new readIndex
  }
  RG_FN void become_follower(uint64_t t, uint64_t l) {
    role = FOLLOWER;
    reset(t);
    leader = l;
  }
  RG_FN void become_candidate() {
    role = CANDIDATE;
    reset(term + 1);
    leader = 0;
    vote = my_id();
  }

  // remote.tryUpdate
  RG_FN bool remote_try_update(uint32_t f, uint64_t idx) {
    const uint64_t nx = RG_GET(rn, f), mt = RG_GET(rm, f);
    const uint32_t st = RG_GET(rt, f);
    if (nx < idx + 1) RG_SET(rn, f, idx + 1);
    if (mt < idx) {
      if (st == WAIT) RG_SET(rt, f, (uint32_t)RETRY);
      RG_SET(rm, f, idx);
      return true;
    }
    return false;
  }

  // raft.tryCommit: q = max{m_i : #{j : m_j >= m_i} >= quorum} = sorted_asc[R - quorum]
  RG_FN bool try_commit() {  // over the voting members only
    uint64_t qv = 0;
    const uint32_t qn = quorum();
    sfor<0, R>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      uint32_t cnt = 0;
      sfor<0, R>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        cnt += ((members >> j) & 1u) && rm[j] >= rm[i] ? 1u : 0u;
      });
      if (((members >> i) & 1u) && cnt >= qn) qv = umax64(qv, rm[i]);
    });
    if (qv > committed && term_at(qv) == term) {
      committed = qv;
      cmv = true;
      return true;
    }
    return false;
  }

  // ---- log writes: term ring + info banks, and a job for the bulk kernel
  // Entry e in [e0, n) goes to index base+e with ring word `word` | (the inline word mt[e·G] of a
  // Replicate or remote Propose, when mt is set) | (len_bits of slab Cmd e, li[e].y, when li is set).
  // Its Cmd bytes go to this replica's payload stream at hw (back to back, whole chunks), and hw
  // advances. aux: a WIRE job's record offset. uspos: a uniform Replicate's (mt and li unset, kind
  // RING) stream position of message entry 0 at the sender, or a caller batch's (kind CMD) arena
  // chunk of entry 0, ucmd = the batch is contiguous in its arena (rg_propose decides).
  RG_FN void write_entries(uint64_t base, uint32_t e0, uint32_t n, uint32_t kind, uint32_t src,
                           const uint64_t* mt, uint64_t word, uint64_t aux = 0, const uint2* li = nullptr,
                           uint32_t uspos = 0, bool ucmd = false) {
    RG_T0(t0);
    write_entries_(base, e0, n, kind, src, mt, word, aux, li, uspos, ucmd);
    RG_ACC(3, t0);
  }
  // FAST: the only log write of the fast path — n entries at fresh indices (past every index read or
  // sent this step: bank 0, nothing to flip), all holding one ring word (a leader's synthetic batch, its
  // no-op, a follower's uniform Replicate from this rank or over the wire), as one uniform job.
  // spos: a RING job's stream position of entry 0 at the sender, a WIRE job's record offset (the job
  // write_entries would make for the same entries)
  RG_FN void write_fresh_uniform(uint64_t base, uint32_t n, uint32_t kind, uint32_t src, uint64_t word,
                                 uint64_t spos) {
#ifdef RG_CTL_FASTREP
    la_n = 0;
#endif
    wlo = umin64(wlo, base);
    const uint32_t ncu = word_nc(word), tot = ncu * n;
    if (n) lt_set(base + n - 1, word & TERM_MASK);
    uint64_t* dst = tr_at(base);
    uint32_t slot = (uint32_t)(base & (P().L - 1));
    const uint64_t step = P().nrep, wrap = (uint64_t)P().L * P().nrep, wr = word & ~BANK_BIT;
    for (uint32_t e = 0; e < n; ++e) {
      *dst = wr;
      dst += step;
      if (++slot == P().L) {
        slot = 0;
        dst -= wrap;
      }
    }
    const bool uni = ncu <= (P().P >> 4);
    if (nj < P().J) {
      const uint64_t n64 = P().nrep, JN = (uint64_t)P().J * n64;
      uint64_t* j64 = P().job64 + (uint64_t)nj * n64 + q;
      j64[J_FIRST * JN] = base;
      j64[J_SPOS * JN] = kind == SRC_RING || kind == SRC_WIRE ? spos : 0ull;
      j64[J_SMASK * JN] = (word & BANK_BIT) ? (n >= 64 ? ~0ull : (1ull << n) - 1) : 0ull;
      j64[J_DMASK * JN] = 0;
      uint32_t* j32 = P().job32 + (uint64_t)nj * n64 + q;
      j32[J_META * JN] = job_meta(n, 0, kind, uni, uni ? ncu : 0u);
      j32[J_SRC * JN] = src;
      j32[J_DPOS * JN] = hw;
      nj++;
    }
    hw += tot;
  }

  RG_FN void write_entries_(uint64_t base, uint32_t e0, uint32_t n, uint32_t kind, uint32_t src,
                            const uint64_t* mt, uint64_t word, uint64_t aux, const uint2* li, uint32_t uspos,
                            bool ucmd) {
    if constexpr (FAST) {  // the fast path writes through write_fresh_uniform only
      (void)base; (void)e0; (void)n; (void)kind; (void)src; (void)mt; (void)word; (void)aux; (void)li;
      (void)uspos; (void)ucmd;
      abort_();
      return;
    } else {
    const uint64_t hi_prot = umax64(last_start, sent_hi);
#ifdef RG_CTL_FASTREP
    la_n = 0;
#endif
    wlo = umin64(wlo, base + e0);
    uint64_t dm = 0, sm = 0, tm = 0;
    // stream layout: tot chunks in all; uniform = every entry the same chunk count ncu (and, for caller
    // Cmds, contiguous in their arena) so the bulk kernel addresses them arithmetically
    uint32_t tot = 0, ncu = 0;
    bool same = true;
#ifdef RG_CTL_FRESH
    if (base + e0 > hi_prot) {
      // Fast path (the steady state): every index is fresh — bank 0, no old word to load, no hull.
      // The ring slot advances by one row per entry (pointer increment, wrap at L) instead of a
      // 64-bit multiply per entry; masks from the words with single-bit selects. (A lane steps one
      // replica; at occupancy 1 this loop is issue-bound)
      uint64_t* dst = tr_at(base + e0);
      uint32_t slot = (uint32_t)((base + e0) & (P().L - 1));
      const uint64_t step = P().nrep, wrap = (uint64_t)P().L * P().nrep;
      if (!mt && !li) {  // one word for every entry: a leader's batch of synthetic Cmds, or its no-op
        const uint64_t M = (n - e0 >= 64 ? ~0ull : (1ull << (n - e0)) - 1) << e0;
        sm = (word & BANK_BIT) ? M : 0ull;
        tm = (word & TYPE_BIT) ? M : 0ull;
        ncu = word_nc(word);
        tot = ncu * (n - e0);
        const uint64_t wr = word & ~BANK_BIT;
        if (n > e0) lt_set(base + n - 1, word & TERM_MASK);
        for (uint32_t e = e0; e < n; ++e) {
          *dst = wr;
          dst += step;
          if (++slot == P().L) {
            slot = 0;
            dst -= wrap;
          }
        }
      } else {
        uint64_t bit = 1ull << e0;
        for (uint32_t e = e0; e < n; e += CB) {
          uint64_t wv[CB];
#pragma unroll
          for (uint32_t k = 0; k < CB; ++k)
            wv[k] = word | (e + k >= n ? 0ull : mt ? mt[(uint64_t)(e + k) * P().G] : len_bits(li[e + k].y));
#pragma unroll
          for (uint32_t k = 0; k < CB; ++k) {
            if (e + k >= n) break;
            const uint64_t w = wv[k];
            if (e + k == n - 1) lt_set(base + n - 1, w & TERM_MASK);
            const uint32_t nc = word_nc(w);
            if (e + k == e0) ncu = nc;
            same = same && nc == ncu;
            tot += nc;
            sm |= (w & BANK_BIT) ? bit : 0ull;
            tm |= (w & TYPE_BIT) ? bit : 0ull;
            *dst = w & ~BANK_BIT;
            dst += step;
            if (++slot == P().L) {
              slot = 0;
              dst -= wrap;
            }
            bit <<= 1;
          }
        }
      }
    } else
#endif
    // CB entries at a time: their loads (sender terms, current ring words of protected
    // indices) are issued before any of their stores, so a lane waits one memory latency per
    // batch instead of one per entry (the compiler cannot prove the ring and the inbox disjoint).
    // The entries of one call occupy distinct ring slots (n <= L by the capacity rule).
    for (uint32_t e = e0; e < n; e += CB) {
      uint64_t wv[CB], ov[CB];
#pragma unroll
      for (uint32_t k = 0; k < CB; ++k) {
        const uint64_t idx = base + e + k;
        const bool in = e + k < n;
        wv[k] = word | (!in ? 0ull : mt ? mt[(uint64_t)(e + k) * P().G] : li ? len_bits(li[e + k].y) : 0ull);
        ov[k] = in && idx <= hi_prot ? *tr_at(idx) : 0;
      }
#pragma unroll
      for (uint32_t k = 0; k < CB; ++k) {
        if (e + k >= n) break;
        const uint32_t ek = e + k;
        const uint64_t idx = base + ek, w = wv[k];
        if (ek == n - 1) lt_set(idx, w & TERM_MASK);
        const uint32_t nc = word_nc(w);
        if (ek == e0) ncu = nc;
        same = same && nc == ncu;
        tot += nc;
        uint32_t tb = 0;
        if (idx <= hi_prot) {  // protected this tick: rewrite goes to the other info bank
          const uint32_t cur = (uint32_t)(ov[k] >> 63);
          const bool in_rw = idx >= rw_lo && idx <= rw_hi;
          tb = in_rw ? cur : cur ^ 1u;
        }
        sm |= (w >> 63) << ek;
        tm |= ((w >> 61) & 1ull) << ek;
        dm |= (uint64_t)tb << ek;
        *tr_at(idx) = (w & ~BANK_BIT) | ((uint64_t)tb << 63);
      }
    }
    const uint64_t lo_w = base + e0, hi_w = umin64(base + n - 1, hi_prot);
    if (lo_w <= hi_w) {
      if (rw_lo > rw_hi) {
        rw_lo = lo_w;
        rw_hi = hi_w;
      } else {
        for (uint64_t i = hi_w + 1; i < rw_lo; ++i) *tr_at(i) ^= BANK_BIT;  // gap below the hull
        rw_lo = umin64(rw_lo, lo_w);
        rw_hi = umax64(rw_hi, hi_w);
      }
    }
    if (tm) cc_hi = umax64(cc_hi, base + n - 1);  // a ConfigChange entry may be among them
    // uniform job? (then J_SPOS = the source position of entry e0's bytes, see raftgpu_internal.h)
    uint64_t spos = 0;
    bool uni = same;
    if (kind == SRC_RING) {
      uni = !mt && !li;  // a uniform Replicate: the sender's stream holds them back to back
      spos = uspos;
    } else if (kind == SRC_WIRE || kind == SRC_WIRE_PROP) {
      uni = same && e0 == 0;  // payloads at +16n + e·ncu chunks
      spos = aux;
    } else if (kind == SRC_CMD) {
      uni = same && ucmd;
      spos = uspos;
    } else {
      uni = true;  // SRC_SLAB (generator Cmds, P bytes) or SRC_NONE (no Cmd bytes)
    }
    uni = uni && ncu <= (P().P >> 4);  // the pipelined path moves at most one lane group (P bytes) per entry
    if (nj < P().J) {
      const uint64_t n64 = P().nrep, JN = (uint64_t)P().J * n64;
      uint64_t* j64 = P().job64 + (uint64_t)nj * n64 + q;
      j64[J_FIRST * JN] = base;
      j64[J_SPOS * JN] = spos;
      j64[J_SMASK * JN] = sm;
      j64[J_DMASK * JN] = dm;
      uint32_t* j32 = P().job32 + (uint64_t)nj * n64 + q;
      j32[J_META * JN] = job_meta(n, e0, kind, uni, uni ? ncu : 0u);
      j32[J_SRC * JN] = src;
      j32[J_DPOS * JN] = hw;
      nj++;
    }
    hw += tot;
    }
  }

  RG_FN uint32_t lpg() const { return lpg_; }

  // raft.appendEntries (leader side): n entries at term. slab_id < 0: the leader's empty no-op.
  // Otherwise Cmds of a proposal: in slab `slab_id`, row of replica slot `rslot` in this column,
  // with lengths li[0..n) (li NULL: synthetic Cmds, P bytes each; li[0].x & SYN_OFF: the generator's
  // Cmds forwarded from that row; else caller Cmds in the slab's arena), or — rmt set: forwarded from
  // another rank — their inline words rmt[e·G] (length bits) and bytes in the receive buffer at
  // record offset wofs. cinfo (a Propose's header word 4): the batch's stream chunks | contiguous in
  // its Cmd arena << 31 | arena chunk of entry 0 << 32. Refused (false) by the ring or the stream
  // capacity rule.
  RG_FN bool append_local(uint32_t n, int slab_id, uint32_t rslot = 0, const uint2* li = nullptr,
                          const uint64_t* rmt = nullptr, uint64_t wofs = 0, uint32_t cc = 0, uint64_t cinfo = 0) {
    if constexpr (FAST) {  // the fast path appends synthetic batches only (caller / forwarded Cmds, changes: full)
      if (cc || rmt || li) {
        abort_();
        return false;
      }
    }
    if (last + n > cap_base + P().L) return false;
    const uint64_t base = last + 1;
    if (cc) {  // one ConfigChange entry: no Cmd, the descriptor in its length field
      write_entries(base, 0, 1, SRC_NONE, 0, nullptr, term | TYPE_BIT | cc_bits(cc));
      last += 1;
      remote_try_update(s, last);
      if (__builtin_popcount(members) == 1) try_commit();  // isSingleNodeQuorum
      return true;
    }
    const bool pay = slab_id >= 0 && P().P;
    if (pay && !stream_fits(hw, lpg(), (uint32_t)cinfo & 0x7FFFFFFFu, P().PTS)) return false;
#ifdef RG_CTL_FASTREP
    const bool plain = base > umax64(last_start, sent_hi);  // no protected index: every bank bit 0
    const uint64_t pt = plain ? term_at(last) : 0;
    const uint32_t pos0 = hw;
#endif
    const bool syn = pay && !rmt && (!li || (li[0].x & SYN_OFF));  // generator Cmds: P bytes each
    const uint64_t w = syn ? term | len_bits(P().P) : term;
    if constexpr (FAST) {
      if (!plain) {
        abort_();
        return false;
      }
      if (!pay) write_fresh_uniform(base, n, SRC_NONE, 0, w, 0);
      else write_fresh_uniform(base, n, SRC_SLAB, (uint32_t)slab_id | (rslot << 16), w, 0);
    } else
    if (!pay) write_entries(base, 0, n, SRC_NONE, 0, nullptr, w);
    else if (rmt) write_entries(base, 0, n, SRC_WIRE_PROP, n, rmt, w, wofs);
    else if (syn) write_entries(base, 0, n, SRC_SLAB, (uint32_t)slab_id | (rslot << 16), nullptr, w);
    else
      write_entries(base, 0, n, SRC_CMD, (uint32_t)slab_id | (rslot << 16), nullptr, w, 0, li, (uint32_t)(cinfo >> 32),
                    (cinfo >> 31) & 1u);
#ifdef RG_CTL_FASTREP
    if (plain && (syn || !pay)) {  // every entry holds the same word
      la_base = base;
      la_word = w;
      la_pt = pt;
      la_n = n;
      la_pos = pos0;
    }
#endif
    last += n;
    remote_try_update(s, last);
    if (__builtin_popcount(members) == 1) try_commit();  // isSingleNodeQuorum
    return true;
  }
  RG_FN void become_leader() {
    role = LEADER;
    reset(term);
    leader = my_id();
    // preLeaderPromotionHandleConfigChange: a ConfigChange entry in (committed, last] is in flight
    for (uint64_t i = committed + 1; i <= umin64(last, cc_hi); ++i)
      if (*tr_at(i) & TYPE_BIT) cc_pending = 1;
    if (!append_local(1, -1)) err |= ERR_RING;  // the empty no-op
  }

  // ---- replication (A.12)
  RG_FN void send_replicate(uint32_t to) {
    const uint32_t st = RG_GET(rt, to);
    if (st == WAIT || st == SNAPSHOT) return;
    const uint64_t next = RG_GET(rn, to);
    if (next <= marker) {  // compacted: InstallSnapshot
      if constexpr (FAST) {
        abort_();
        return;
      }
      if (!(active & (1u << to))) return;
      if (snap_index == 0) {
        err |= ERR_EMPTY_SNAP;
        return;
      }
      rs_set(to, snap_index);
      RG_SET(rt, to, (uint32_t)SNAPSHOT);
      send(M_INSTALL_SNAPSHOT, to + 1, 0, 0, 0, snap_term, snap_index, 0, 0, snap_members, 0, 0);
      return;
    }
    const uint32_t n = next <= last ? (uint32_t)umin64(P().E, last - next + 1) : 0;
#ifdef RG_CTL_FASTREP  // the whole message lies in this step's plain append (the steady-state case)
    // (at R >= 7 the three extra live registers push the lane past 512 and into scratch: off there)
    const bool fast = R <= 6 && n > 0 && la_n > 0 && next >= la_base && next + n <= la_base + la_n;
    const uint64_t lt = !fast ? term_at(next - 1) : next == la_base ? la_pt : la_word & TERM_MASK;
    if constexpr (FAST) {  // entries read back from the ring (a lagging follower): the full step's
      if (n > 0 && !fast) {
        abort_();
        return;
      }
    }
#else
    const uint64_t lt = term_at(next - 1);
#endif
    if (n > 0) {  // remote.progress
      if (st == REPLICATE) RG_SET(rn, to, next + n);
      else if (st == RETRY) RG_SET(rt, to, (uint32_t)WAIT);
    }
#ifdef RG_CTL_FASTREP
    const uint32_t uni = fast ? RG_UNIFORM : 0u;
    // a uniform Replicate's word 5: the stream position of its first entry's Cmd here (the
    // follower's bulk job reads the bytes from there; shown as hint 0 by rg_read_msgs)
    const uint64_t upos = fast ? (uint32_t)(la_pos + (uint32_t)(next - la_base) * word_nc(la_word)) : 0u;
#else
    const uint32_t uni = 0;
    const uint64_t upos = 0;
#endif
    const int k = send(M_REPLICATE, to + 1, 0, 0, n, lt, next - 1, committed, upos, 0, uni, 0);
    if (k >= 0 && n > 0) {
      uint64_t* mt = P().mt_out + ((((uint64_t)RG_S_SEND * R + to) * P().K + (uint32_t)k) * P().E) * P().G + g;
#ifdef RG_CTL_FASTREP
      if (FAST || fast) {
        mt[0] = la_word;  // uniform: one word for every entry
      } else
#endif
      for (uint32_t e = 0; e < n; e += CB) {  // term|type|pay|bank; batched as in write_entries
        uint64_t v[CB];
#pragma unroll
        for (uint32_t k2 = 0; k2 < CB; ++k2) v[k2] = e + k2 < n ? *tr_at(next + e + k2) : 0;
#pragma unroll
        for (uint32_t k2 = 0; k2 < CB; ++k2)
          if (e + k2 < n) mt[(uint64_t)(e + k2) * P().G] = v[k2];
      }
      sent_hi = umax64(sent_hi, next + n - 1);
    }
  }
  RG_FN void broadcast_replicate() {
    for (uint32_t i = 0; i < R; ++i) {
      if (i != s && is_member(i)) send_replicate(i);
      if (FAST && aborted) return;
    }
  }
  RG_FN void broadcast_heartbeat() {
    // the newest pending ReadIndex rides on every heartbeat (dragonboat's broadcastHeartbeatMessage
    // attaches readIndex.peepCtx), so a lost read heartbeat or response is retried by the next round
    uint64_t ctx = 0;
    if (P().rdst) {
      const uint64_t nq = umin64(P().rdst[(uint64_t)RQ_N * P().nrep + q], RG_RQ);
      if (nq) ctx = P().rdst[(RQ_CTX + nq - 1) * (uint64_t)P().nrep + q];
    }
    if constexpr (FAST) {  // a pending read: its confirmation round is the full step's
      if (ctx) {
        abort_();
        return;
      }
    }
    for (uint32_t i = 0; i < R; ++i)
      if (i != s && is_member(i)) send(M_HEARTBEAT, i + 1, 0, 0, 0, 0, 0, umin64(RG_GET(rm, i), committed), ctx, 0, 0, 0);
  }

  // ---- follower side (A.9)
  // remote: the message came over the wire (its inline terms are in rmt, its records at wofs)
  // upos: header word 5 (a uniform Replicate's stream position of entry 0 at the sender)
  RG_FN void handle_replicate(uint64_t w0, uint64_t log_term, uint64_t li, uint64_t mcommit, uint32_t from,
                              uint32_t src, uint32_t k, bool remote, uint64_t wofs, uint64_t upos, uint64_t mt0) {
    RG_T0(t0);
    handle_replicate_(w0, log_term, li, mcommit, from, src, k, remote, wofs, upos, mt0);
    RG_ACC(2, t0);
  }
  RG_FN void handle_replicate_(uint64_t w0, uint64_t log_term, uint64_t li, uint64_t mcommit, uint32_t from,
                               uint32_t src, uint32_t k, bool remote, uint64_t wofs, uint64_t upos, uint64_t mt0) {
    if (li < committed) {
      send_simple(M_REPLICATE_RESP, from, 0, committed);
      return;
    }
    const uint32_t n = (uint32_t)(w0 >> 32);
    // a remote Replicate's word 7 is its records' offset in the receive buffer (16-B aligned), with
    // RG_UNIFORM set by unpack_kernel when every entry record holds the same application ring word
    const bool runi = remote && ((uint32_t)wofs & RG_UNIFORM) && n > 0;
    // a uniform Replicate: every entry carries the word mt[0] (local: the sender wrote only that one)
    const bool uni = !remote && ((uint32_t)wofs & RG_UNIFORM) && n > 0;
    wofs &= ~(uint64_t)RG_UNIFORM;
    if (term_at(li) == log_term) {
      const uint64_t* mt = (remote ? P().rmt : P().mt_in) + ((((uint64_t)src * R + RG_S_INBOX) * P().K + k) * P().E) * P().G + g;
      const uint64_t uw = uni || runi ? mt0 : 0ull;  // loaded with the header (handle_)
      if constexpr (FAST) {  // an append at the log end from a uniform Replicate (or an empty one)
        if (li != last || (n > 0 && !uni && !runi) || (uw & TYPE_BIT)) {
          abort_();
          return;
        }
        const uint64_t last_new = li + n;
        if (n > 0) {  // every index is new: no conflict scan (entryLog.getConflictIndex finds li + 1)
          if (last_new > cap_base + P().L || (P().P && !stream_fits(hw, lpg(), n * word_nc(uw), P().PTS))) {
            drops++;  // capacity rules (ring, then payload stream): dropped, no reply
            return;
          }
          if (li + 1 <= umax64(last_start, sent_hi)) {
            abort_();
            return;
          }
          if (remote) write_fresh_uniform(li + 1, n, SRC_WIRE, n, uw, wofs);
          else write_fresh_uniform(li + 1, n, SRC_RING, src * P().G + g, uw, (uint32_t)upos);
          last = last_new;
        }
        commit_to(umin64(last_new, mcommit));
        if (aborted) return;
        send_simple(M_REPLICATE_RESP, from, 0, last_new);
        return;
      }
      uint32_t k0 = n;
      for (uint32_t e = 0; e < n; ++e) {  // entryLog.getConflictIndex
        if (term_at(li + 1 + e) != ((uni ? uw : mt[(uint64_t)e * P().G]) & TERM_MASK)) {
          k0 = e;
          break;
        }
      }
      const uint64_t last_new = li + n;
      if (k0 < n) {
        const uint64_t ci = li + 1 + k0;
        if (ci > committed) {  // capacity rules (ring, then payload stream): dropped, no reply
          bool fits = last_new <= cap_base + P().L;
          if (fits && P().P) {
            uint32_t c = 0;
            if (uni) c = (n - k0) * word_nc(uw);
            else
              for (uint32_t e = k0; e < n; ++e) c += word_nc(mt[(uint64_t)e * P().G]);
            fits = stream_fits(hw, lpg(), c, P().PTS);
          }
          if (!fits) {
            drops++;
            return;
          }
        }
        if (ci <= committed) {
          err |= ERR_CONFLICT;
        } else {
          if (remote) write_entries(li + 1, k0, n, SRC_WIRE, n, mt, 0, wofs);
          else if (uni) write_entries(li + 1, k0, n, SRC_RING, src * P().G + g, nullptr, uw, 0, nullptr, (uint32_t)upos);
          else write_entries(li + 1, k0, n, SRC_RING, src * P().G + g, mt, 0);
          last = last_new;
        }
      }
      commit_to(umin64(last_new, mcommit));
      send_simple(M_REPLICATE_RESP, from, 0, last_new);
    } else {
      send_simple(M_REPLICATE_RESP, from, 1, li, last);
    }
  }

  RG_FN void handle_install_snapshot(uint64_t si, uint64_t stt, uint32_t from, uint32_t smembers) {
    uint64_t li;
    if (si <= committed) {
      li = committed;
    } else if (term_at(si) == stt) {
      commit_to(si);
      li = committed;
    } else {  // restore; the state machine recovers from the snapshot
      marker = last = committed = snap_index = processed = si;
      applied = umax64(applied, si);
#ifdef RG_CTL_FASTREP
      la_n = 0;
#endif
      marker_term = snap_term = stt;
      members = snap_members = smembers;  // the snapshot's membership
      li = last;
      restored_at = si;
    }
    send_simple(M_REPLICATE_RESP, from, 0, li);
  }

  // ---- elections (A.7, A.8)
  RG_FN void campaign() {
    become_candidate();
    responded |= 1u << s;
    granted |= 1u << s;
    if ((uint32_t)__builtin_popcount(granted & members) == quorum()) {  // single-node quorum
      become_leader();
      return;
    }
    const uint64_t lt = term_at(last);
    for (uint32_t i = 0; i < R; ++i)
      if (i != s && is_member(i)) send(M_REQUEST_VOTE, i + 1, term, 0, 0, lt, last, 0, 0, 0, 0, 0);
  }
  RG_FN void handle_node_election() {
    if (role == LEADER) return;
    if (!is_member(s)) return;        // selfRemoved: no elections
    if (committed > applied) return;  // hasConfigChangeToApply
    if (term >= TERM_MASK) {          // the next term would not fit the ring word's 36-bit field
      err |= ERR_TERM;
      return;
    }
    campaign();
  }
  RG_FN void handle_request_vote(uint64_t log_term, uint64_t log_index, uint32_t from) {
    const bool can = vote == 0 || vote == from;
    const uint64_t lt = term_at(last);
    const bool utd = log_term > lt || (log_term == lt && log_index >= last);
    uint32_t rej = 1;
    if (can && utd) {
      etick = 0;
      vote = from;
      rej = 0;
    }
    send_simple(M_REQUEST_VOTE_RESP, from, rej);
  }
  RG_FN void candidate_vote_resp(uint32_t from, uint32_t reject) {
    const uint32_t bit = 1u << (from - 1);
    if (!(responded & bit)) {
      responded |= bit;
      if (!reject) granted |= bit;
    }
    const uint32_t gr = __builtin_popcount(granted & members), tot = __builtin_popcount(responded & members);
    if (gr == quorum()) {
      become_leader();
      broadcast_replicate();
    } else if (tot - gr == quorum()) {
      become_follower(term, 0);
    }
  }

  // ---- leader responses (A.10, A.11)
  RG_FN void leader_replicate_resp(uint32_t reject, uint64_t li, uint64_t hint, uint32_t from) {
    const uint32_t f = from - 1;
    if (!is_member(f)) return;  // no remote for it
    if constexpr (FAST) {  // a rejection walks the remote back (decreaseTo), a snapshot remote: the full step's
      if (reject || RG_GET(rt, f) == SNAPSHOT) {
        abort_();
        return;
      }
    }
    active |= 1u << f;
    if (!reject) {
      const uint32_t st0 = RG_GET(rt, f);
      const bool paused = st0 == WAIT || st0 == SNAPSHOT;
      if (remote_try_update(f, li)) {
        const uint32_t st = RG_GET(rt, f);
        const uint64_t m = RG_GET(rm, f), sn = rs_get(f);
        if (st == RETRY) {  // respondedTo → becomeReplicate
          RG_SET(rn, f, m + 1);
          rs_set(f, 0ull);
          RG_SET(rt, f, (uint32_t)REPLICATE);
        } else if (st == SNAPSHOT && m >= sn) {  // becomeRetry from Snapshot
          RG_SET(rn, f, umax64(m + 1, sn + 1));
          rs_set(f, 0ull);
          RG_SET(rt, f, (uint32_t)RETRY);
        }
        if (try_commit()) broadcast_replicate();
        else if (paused) send_replicate(f);
      }
    } else {  // remote.decreaseTo
      const uint32_t st = RG_GET(rt, f);
      const uint64_t m = RG_GET(rm, f), nx = RG_GET(rn, f);
      bool ok;
      if (st == REPLICATE) {
        if (li <= m) ok = false;
        else {
          RG_SET(rn, f, m + 1);
          ok = true;
        }
      } else if (nx - 1 != li) {
        ok = false;
      } else {
        if (st == WAIT) RG_SET(rt, f, (uint32_t)RETRY);
        RG_SET(rn, f, umax64(1, umin64(li, hint + 1)));
        ok = true;
      }
      if (ok) {
        if (RG_GET(rt, f) == REPLICATE) {  // enterRetryState → becomeRetry
          RG_SET(rn, f, m + 1);
          rs_set(f, 0ull);
          RG_SET(rt, f, (uint32_t)RETRY);
        }
        send_replicate(f);
      }
    }
  }
  RG_FN void leader_heartbeat_resp(uint32_t from, uint64_t hint) {
    const uint32_t f = from - 1;
    if (!is_member(f)) return;  // no remote for it
    if constexpr (FAST) {  // a read heartbeat's answer (readIndex.confirm): the full step's
      if (hint != 0) {
        abort_();
        return;
      }
    }
    active |= 1u << f;
    if (RG_GET(rt, f) == WAIT) RG_SET(rt, f, (uint32_t)RETRY);
    if (RG_GET(rm, f) < last) send_replicate(f);
    if (hint != 0 && P().rdst) read_confirm(hint, f);  // only read heartbeats carry a context
  }
  // readIndex.confirm: the request this heartbeat answered; once a quorum confirmed it, it and every
  // request queued before it are done, all at its index (dragonboat rewrites v.index = s.index)
  RG_FN void read_confirm(uint64_t hint, uint32_t f) {
    uint64_t* rd = P().rdst + q;
    const uint64_t n = P().nrep;
    const uint32_t nq = (uint32_t)umin64(rd[RQ_N * n], RG_RQ);  // rows written only here: <= RG_RQ
    uint32_t k = 0;
    while (k < nq && rd[(RQ_CTX + k) * n] != hint) ++k;
    if (k == nq) return;
    const uint64_t a = rd[(RQ_ACKS + k) * n] | (1ull << f);
    if ((uint32_t)__builtin_popcount((uint32_t)a & members) < quorum()) {
      rd[(RQ_ACKS + k) * n] = a;
      return;
    }
    const uint64_t index = rd[(RQ_INDEX + k) * n];
    uint64_t ctx[RG_RQ], acks[RG_RQ];
    for (uint32_t i = 0; i <= k; ++i) {
      ctx[i] = rd[(RQ_CTX + i) * n];
      acks[i] = rd[(RQ_ACKS + i) * n];
    }
    for (uint32_t i = k + 1; i < nq; ++i) {  // the rest move to the front
      rd[(RQ_CTX + i - k - 1) * n] = rd[(RQ_CTX + i) * n];
      rd[(RQ_INDEX + i - k - 1) * n] = rd[(RQ_INDEX + i) * n];
      rd[(RQ_ACKS + i - k - 1) * n] = rd[(RQ_ACKS + i) * n];
    }
    rd[RQ_N * n] = nq - k - 1;
    for (uint32_t i = 0; i <= k; ++i) read_confirmed(ctx[i], index, (uint32_t)(acks[i] >> 32));
  }
  // ---- ReadIndex (Raft thesis §6.4; dragonboat's readIndex), state in P().rdst, not in registers
  RG_FN void read_ready(uint64_t ctx, uint64_t index) {  // addReadyToRead, at most RG_RQ per step
    uint64_t* rd = P().rdst + q;
    const uint64_t n = P().nrep;
    uint64_t k = umin64(rd[RD_N * n], RG_RQ);
    if (rd[RD_TICK * n] != P().tick + 1) {  // the first read made ready in this step
      rd[RD_TICK * n] = P().tick + 1;
      k = 0;
    }
    if (k == RG_RQ) {  // the step's ready list is full: dropped (counted)
      drops++;
      return;
    }
    rd[(RD_CTX + k) * n] = ctx;
    rd[(RD_INDEX + k) * n] = index;
    rd[RD_N * n] = k + 1;
  }
  RG_FN void read_confirmed(uint64_t ctx, uint64_t index, uint32_t slot) {
    if (slot == s) read_ready(ctx, index);
    else send(M_READ_INDEX_RESP, slot + 1, 0, 0, 0, 0, index, 0, ctx, 0, 0, 0);
  }
  RG_FN void handle_read_index(uint32_t from, uint64_t ctx) {
    const uint32_t f = from - 1;
    if (!P().rdst) return;
    if (role == LEADER) {
      uint64_t* rd = P().rdst + q;
      const uint64_t n = P().nrep;
      if (quorum() == 1) {  // isSingleNodeQuorum
        read_confirmed(ctx, committed, f);
      } else if (term_at(committed) != term) {
        drops++;  // nothing committed in this term yet (thesis §6.4)
      } else {
        const uint32_t nq = (uint32_t)umin64(rd[RQ_N * n], RG_RQ);
        uint32_t k = 0;  // readIndex.addRequest: a context already pending is not added again
        while (k < nq && rd[(RQ_CTX + k) * n] != ctx) ++k;
        if (k == nq) {
          if (nq == RG_RQ) {  // the queue is full: dropped (counted), no heartbeat
            drops++;
            return;
          }
          rd[(RQ_CTX + k) * n] = ctx;
          rd[(RQ_INDEX + k) * n] = committed;
          rd[(RQ_ACKS + k) * n] = (1ull << s) | ((uint64_t)f << 32);
          rd[RQ_N * n] = nq + 1;
        }
        for (uint32_t i = 0; i < R; ++i)  // broadcastHeartbeatMessageWithHint
          if (i != s && is_member(i)) send(M_HEARTBEAT, i + 1, 0, 0, 0, 0, 0, umin64(RG_GET(rm, i), committed), ctx, 0, 0, 0);
      }
    } else if (role == FOLLOWER && leader != 0 && f == s) {
      send(M_READ_INDEX, (uint32_t)leader, 0, 0, 0, 0, 0, 0, ctx, 0, 0, 0);
    } else {
      drops++;
    }
  }
  RG_FN void check_quorum() {
    const uint32_t c = __builtin_popcount((active | (1u << s)) & members);  // leaderHasQuorum
    if constexpr (FAST) {  // stepping down: the full step's
      if (c < quorum()) {
        abort_();
        return;
      }
      active = 0;
    } else {
      active = 0;
      if (c < quorum()) become_follower(term, 0);
    }
  }

  // ---- proposals: nent Cmds (hm = those with a non-empty Cmd, the forwarded header's hint); their
  // bytes and lengths as append_local takes them
  // cc != 0: a membership change (one ConfigChange entry)
  RG_FN void handle_propose(uint32_t nent, uint32_t slab_id, uint32_t hop, uint64_t hm, uint32_t rslot,
                            const uint2* li, const uint64_t* rmt, uint64_t wofs, uint32_t cc, uint64_t cinfo) {
    if constexpr (FAST) {  // forwarding, dropping at a candidate, membership changes: the full step's
      if (role != LEADER || cc) {
        abort_();
        return;
      }
    }
    if (role == LEADER) {
      RG_T0(t0);
      const bool dropped = cc && cc_pending;  // one change at a time: an empty entry instead
      if (!(cc ? (dropped ? append_local(1, -1) : append_local(1, -1, 0, nullptr, nullptr, 0, cc))
               : append_local(nent, (int)slab_id, rslot, li, rmt, wofs, 0, cinfo))) {
        drops++;
        return;
      }
      if (FAST && aborted) return;
      if (dropped) drops++;        // reportDroppedConfigChange
      else if (cc) cc_pending = 1;  // setPendingConfigChange
      RG_ACC(0, t0);
      RG_T0(t1);
      broadcast_replicate();
      RG_ACC(1, t1);
    } else if (role == FOLLOWER && leader != 0 && hop == 0) {
      send(M_PROPOSE, (uint32_t)leader, 0, 0, nent, 0, 0, cinfo, hm, cc, slab_id, hop + 1);
    } else {
      drops++;
    }
  }

  // ---- timers (A.6)
  RG_FN void tick() {
    if (role == LEADER) {
      etick++;
      if (etick >= P().ET) {
        etick = 0;
        if (P().CQ) check_quorum();
        if (FAST && aborted) return;
      }
      htick++;
      if (htick >= P().HT) {
        htick = 0;
        if (role == LEADER) broadcast_heartbeat();
      }
    } else {
      etick++;
      if (is_member(s) && etick >= rand_to) {  // selfRemoved: no elections
        if constexpr (FAST) {  // a campaign: the full step's
          abort_();
          return;
        }
        etick = 0;
        handle_node_election();
      }
    }
  }

  // ---- membership: raft.addNode / removeNode through the rsm's ApplyConfigChange
  RG_FN void apply_config_change(uint32_t cc) {
    cc_pending = 0;  // clearPendingConfigChange
    const uint32_t op = cc >> 4, slot = (cc & 0xFu) - 1u;
    if (slot >= (uint32_t)R) return;
    const uint32_t bit = 1u << slot;
    if (op == CC_ADD) {
      if (members & bit) return;
      members |= bit;  // setRemote(id, 0, lastIndex + 1)
      RG_SET(rm, slot, 0ull);
      RG_SET(rn, slot, last + 1);
      rs_set(slot, 0ull);
      RG_SET(rt, slot, (uint32_t)RETRY);
    } else if (op == CC_REMOVE) {
      members &= ~bit;  // deleteRemote
      active &= ~bit;
      if (slot == s && role == LEADER) become_follower(term, 0);
      if (role == LEADER && members && try_commit()) broadcast_replicate();
    }
  }

  // ---- Handle (A.3): message k from slot src (remote: it came over the wire from another rank)
  // words 0 and 1 (type, ids, term) up front; the others where a handler uses them
  // (RG_CTL_HDRBATCH: all eight in one round trip; at R >= 6 there is no room for them)
#ifdef RG_CTL_HDRBATCH
  static constexpr int NB = R <= 5 ? 8 : 2;
#else
  static constexpr int NB = 2;
#endif
  struct Hdr {
    uint64_t w[NB];
    uint64_t mt0;  // a Replicate's first inline word (a uniform Replicate needs only it)
  };
  RG_FN const uint64_t* hdr_ptr(uint32_t src, uint32_t k, bool remote) const {
    return (remote ? P().rhdr : P().hdr_in) + (((uint64_t)src * R + RG_S_INBOX) * P().K + k) * P().G + g;
  }
  // one round trip: the header words and the message's first inline word (for other
  // messages the slot holds stale words, which nothing reads)
  // cls: the message's class from the count plane (cnt_cls). The fast step loads only that class's words
  // (and the first inline term only for MC_ALL); the full step loads every word it batches
  RG_FN void load_hdr(uint32_t src, uint32_t k, bool remote, Hdr& o, uint32_t cls = MC_ALL) const {
    const uint64_t plane = (uint64_t)R * R * P().K * P().G;
    const uint64_t* h = hdr_ptr(src, k, remote);
    if constexpr (FAST && NB == 8) {
      uint32_t wm = cls_words(cls);
      // a leader's fast step handles responses only (ids|reject, term, log index, hint); a Replicate or
      // Heartbeat it ignores, any other type leaves the fast path (its words unread)
      if constexpr (ROLE == (int)LEADER) wm &= 0x2Bu;
#pragma unroll
      for (int x = 0; x < NB; ++x) o.w[x] = (wm >> x) & 1u ? h[(uint64_t)x * plane] : 0ull;
      o.mt0 = ROLE != (int)LEADER && cls == MC_ALL
                  ? (remote ? P().rmt : P().mt_in)[((((uint64_t)src * R + RG_S_INBOX) * P().K + k) * P().E) * P().G + g]
                  : 0ull;
      return;
    }
#pragma unroll
    for (int x = 0; x < NB; ++x) o.w[x] = h[(uint64_t)x * plane];
    o.mt0 = (remote ? P().rmt : P().mt_in)[((((uint64_t)src * R + RG_S_INBOX) * P().K + k) * P().E) * P().G + g];
  }
  RG_FN void handle(uint32_t src, uint32_t k, bool remote, const Hdr& hd) {
    RG_T0(t0);
    handle_(src, k, remote, hd);
    RG_ACC(5, t0);
  }
  RG_FN void handle_(uint32_t src, uint32_t k, bool remote, const Hdr& hd) {
    const uint64_t plane = (uint64_t)R * R * P().K * P().G;
    const uint64_t* h = hdr_ptr(src, k, remote);
    const uint64_t mt0 = hd.mt0;
    auto hw = [&](int x) -> uint64_t { return x < NB ? hd.w[x < NB ? x : 0] : h[(uint64_t)x * plane]; };
    const uint64_t w0 = hw(0);
    const uint64_t mterm = hw(1);
    const uint32_t type = (uint32_t)(w0 & 0xFF);
    const uint32_t from = (uint32_t)(w0 >> 8) & 0xFF;
    if constexpr (FAST) {
      // same-term steady-state traffic only, from this rank or over the wire: a term change, a vote, a
      // read, a forwarded proposal or a snapshot leaves the fast path (a candidate never entered it)
#ifdef RG_AB_FAST_NO_REMOTE  // diagnostic variant: r04's fast step, which handed every remote message off
      if (remote) {
        abort_();
        return;
      }
#endif
      if (from - 1 >= (uint32_t)R || (mterm != 0 && mterm != term) ||
          (type == M_REPLICATE && (uint32_t)(w0 >> 32) > P().E)) {
        abort_();
        return;
      }
      switch (type) {
        case M_REPLICATE:
        case M_HEARTBEAT:
          if (role == LEADER) return;  // a leader ignores them (as the full step's dispatch does)
          etick = 0;
          if (leader != from) {  // the first message of a new leader in this term
            leader = from;
            ldv = true;
          }
          if (type == M_REPLICATE) {
            handle_replicate(w0, hw(2), hw(3), hw(4), from, src, k, remote, hw(7), hw(5), mt0);
          } else {
            if (hw(5) || hw(6)) {  // a read heartbeat (its context echoed): the full step's
              abort_();
              return;
            }
            commit_to(hw(4));
            if (aborted) return;
            send_simple(M_HEARTBEAT_RESP, from, 0, 0, 0, 0);
          }
          return;
        case M_REPLICATE_RESP:
          if (role == LEADER) leader_replicate_resp((uint32_t)(w0 >> 24) & 0xFF, hw(3), hw(5), from);
          return;
        case M_HEARTBEAT_RESP:
          if (role == LEADER) leader_heartbeat_resp(from, hw(5));
          return;
        case M_NOOP:
          return;
        default:
          abort_();
          return;
      }
    }
    if (from - 1 >= (uint32_t)R) {  // unreachable: local senders stamp their id, unpack checks remote ones
      err |= ERR_WIRE;
      return;
    }
    // unreachable (senders write at most E entries, unpack_kernel keeps only well-formed messages):
    // checked anyway, so that a damaged inbox shows up as ERR_WIRE instead of a wild address
    if (type == M_REPLICATE && (uint32_t)(w0 >> 32) > P().E) {
      RG_OOB("RG_BOUNDS control q=%u src=%u k=%u remote=%d replicate n=%u > E=%u\n", q, src, k, (int)remote,
             (uint32_t)(w0 >> 32), P().E);
      err |= ERR_WIRE;
      return;
    }
    const bool leader_msg =
        type == M_REPLICATE || type == M_INSTALL_SNAPSHOT || type == M_HEARTBEAT || type == M_READ_INDEX_RESP;
    if (mterm != 0 && mterm != term) {
      if (type == M_REQUEST_VOTE && P().CQ && mterm > term && hw(5) != from && leader != 0 && etick < P().ET)
        return;
      if (mterm > term) {
        become_follower(mterm, leader_msg ? from : 0);
      } else {
        if (P().CQ && leader_msg) send_simple(M_NOOP, from);
        return;
      }
    }
    switch (type) {
      case M_PROPOSE: {  // forwarded (hop 1). Local: the Cmds are in the forwarder's row of slab w7;
        // remote: unpack put their length words in rmt and their records' offset in word 7
        const uint64_t w7 = hw(7);
        const uint32_t nent = (uint32_t)(w0 >> 32);
        if (nent - 1 >= P().E || (!remote && (uint32_t)w7 >= P().nslab)) {  // unreachable: senders forward
          err |= ERR_WIRE;                                               // 1..E entries of a slab
          break;
        }
        // word 4: the batch's stream chunks | contiguous << 31 | arena chunk << 32 (a remote
        // batch: the chunks unpack_kernel counted)
        if (remote) {
          const uint64_t* rm = P().rmt + ((((uint64_t)src * R + RG_S_INBOX) * P().K + k) * P().E) * P().G + g;
          handle_propose(nent, 0, 1, hw(5), 0, nullptr, rm, w7, (uint32_t)hw(6), hw(4));
        } else {
          const uint64_t row = P().wire ? (uint64_t)src * P().G + g : g;  // the forwarder's slab row (same rank)
          const uint64_t rows = P().wire ? P().nrep : P().G;
          const uint2* li = P().slab_info + ((uint64_t)(uint32_t)w7 * rows + row) * P().E;
          handle_propose(nent, (uint32_t)w7, (uint32_t)(w7 >> 32), hw(5), src, li, nullptr, 0, (uint32_t)hw(6), hw(4));
        }
        break;
      }
      case M_REPLICATE:
      case M_HEARTBEAT:
      case M_INSTALL_SNAPSHOT:
        if (role == LEADER) break;
        if (role == CANDIDATE) {
          become_follower(term, from);
        } else {
          etick = 0;
          leader = from;
        }
        if (type == M_REPLICATE) {
          handle_replicate(w0, hw(2), hw(3), hw(4), from, src, k, remote, hw(7), hw(5), mt0);  // local: RG_UNIFORM
        } else if (type == M_HEARTBEAT) {
          commit_to(hw(4));
          send_simple(M_HEARTBEAT_RESP, from, 0, 0, hw(5), hw(6));
        } else {
          handle_install_snapshot(hw(3), hw(2), from, (uint32_t)hw(6));
        }
        break;
      case M_REPLICATE_RESP:
        if (role == LEADER) leader_replicate_resp((uint32_t)(w0 >> 24) & 0xFF, hw(3), hw(5), from);
        break;
      case M_HEARTBEAT_RESP:
        if (role == LEADER) leader_heartbeat_resp(from, hw(5));
        break;
      case M_READ_INDEX:
        handle_read_index(from, hw(5));
        break;
      case M_READ_INDEX_RESP:
        if (role == FOLLOWER && P().rdst) {
          etick = 0;
          leader = from;
          read_ready(hw(5), hw(3));
        }
        break;
      case M_REQUEST_VOTE:
        handle_request_vote(hw(2), hw(3), from);
        break;
      case M_REQUEST_VOTE_RESP:
        if (role == CANDIDATE) candidate_vote_resp(from, (uint32_t)(w0 >> 24) & 0xFF);
        break;
      default:
        break;
    }
  }

  // ---- the whole step
  uint32_t stamps[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};

  // the next inbox header is loaded before the current message is handled (one round trip for the
  // whole inbox), except in the followers' fast step: a follower's inbox is a Replicate and perhaps a
  // Heartbeat, and without the second header live the step fits three waves per SIMD (r04)
#if defined(RG_CTL_FAST_NOPIPE)
  static constexpr bool PIPE = !FAST;
#elif defined(RG_CTL_FAST_PIPE)
  static constexpr bool PIPE = true;
#else
  static constexpr bool PIPE = !(FAST && ROLE == FOLLOWER);
#endif

  RG_FN void run() {
    // The step's inputs that no step logic feeds — the inbox counts of every sender and the tick
    // inputs — are loaded together up front: the lane then waits one memory latency for all of them
    // instead of one per use (at C2 a wave per SIMD, so nothing hides these waits)
    uint32_t cnt_pf[R];
    sfor<0, R>([&](auto jc) {
      constexpr int src = decltype(jc)::value;
      cnt_pf[src] = (uint32_t)src == s ? 0u
                    : (pl_remote(P().pl, src, RG_S_INBOX, g) ? P().rcnt : P().cnt_in)[((uint64_t)src * R + RG_S_INBOX) * P().G + g];
    });
    const uint32_t in_pt = P().prop_target ? P().prop_target[gi] : 0xFFu;
    const uint32_t in_pc = P().prop_target ? P().prop_count[gi] : 0u;
    const bool in_camp = P().campaign && P().campaign[ri()];
    const uint32_t in_cc = P().cc_in ? P().cc_in[gi] : 0u;
    const uint64_t in_rd = P().read_ctx ? P().read_ctx[ri()] : 0ull;
    sfor<0, R>([&](auto jc) {
      constexpr int src = decltype(jc)::value;
      if (cnt_n(cnt_pf[src]) > P().K) {  // never produced by a sender (unpack_kernel clamps received counts): ERR_WIRE
        RG_OOB("RG_BOUNDS control q=%u src=%u cnt=%u > K=%u\n", q, (uint32_t)src, cnt_n(cnt_pf[src]), P().K);
        if constexpr (FAST) abort_();
        err |= ERR_WIRE;
        cnt_pf[src] = 0;
      }
    });
    // The inbox in sender order, software-pipelined: the next message's header is loaded before the
    // current one is handled (the inbox is read-only in this launch), so a lane waits about one
    // round trip for its whole inbox instead of one per message.
    auto next_msg = [&](uint32_t src, uint32_t k, uint32_t& ns, uint32_t& nk) -> bool {
      for (uint32_t x = src, y = k + 1; x < R; ++x, y = 0) {
        if (x == s) continue;
        if (y < cnt_n(sel_get<R>(cnt_pf, x))) {
          ns = x;
          nk = y;
          return true;
        }
      }
      return false;
    };
    uint32_t cs = 0, ck = 0;
    bool have = !(FAST && aborted) && next_msg(0, ~0u, cs, ck);
    Hdr cur{};
    if (have) load_hdr(cs, ck, pl_remote(P().pl, cs, RG_S_INBOX, g), cur, cnt_cls(sel_get<R>(cnt_pf, cs), ck));
    while (have) {
      uint32_t ns = 0, nk = 0;
      const bool more = next_msg(cs, ck, ns, nk);
      Hdr nxt{};
      if (PIPE && more) load_hdr(ns, nk, pl_remote(P().pl, ns, RG_S_INBOX, g), nxt, cnt_cls(sel_get<R>(cnt_pf, ns), nk));
      handle(cs, ck, pl_remote(P().pl, cs, RG_S_INBOX, g), cur);
      if (!PIPE && more && !(FAST && aborted))
        load_hdr(ns, nk, pl_remote(P().pl, ns, RG_S_INBOX, g), nxt, cnt_cls(sel_get<R>(cnt_pf, ns), nk));
      cur = nxt;
      cs = ns;
      ck = nk;
      have = more && !(FAST && aborted);
    }
    RG_STAMP(1);
    if constexpr (FAST) {  // a campaign input, a membership change or a read at this replica: the full step's
      if (in_camp || (in_cc && (in_cc & 0xFFu) == s) || in_rd) abort_();
      if (aborted) return;
    }
    if (in_camp) handle_node_election();
    if (!(P().flags & 1u)) tick();
    if (FAST && aborted) return;
    RG_STAMP(2);
    if (in_pt == s) {
      const uint32_t n = in_pc;
      if (n > P().E) {  // rg_tick_device's contract: batches of at most E entries (the host path checks)
        drops++;
      } else if (n > 0) {
        // caller batch (rg_propose): lengths in slab_info; tick-input batch: synthetic Cmds of P bytes
        const uint32_t sl = (uint32_t)(P().tick % P().nslab);
        const uint64_t row = P().wire ? q : g, rows = P().wire ? P().nrep : P().G;
        const uint64_t hm = !P().P ? 0ull : P().prop_hmask ? P().prop_hmask[gi] : (n >= 64 ? ~0ull : (1ull << n) - 1);
        const uint2* li = P().prop_hmask && P().P ? P().slab_info + ((uint64_t)sl * rows + row) * P().E : nullptr;
        uint64_t cinfo = (uint64_t)(n * (P().P >> 4)) | (1ull << 31);  // generator Cmds: P bytes each
        if (P().prop_cmd) {  // a caller batch: rg_propose's chunk count, contiguity and first arena chunk
          const uint2 pc = P().prop_cmd[gi];
          cinfo = pc.x | ((uint64_t)pc.y << 32);
        }
        handle_propose(n, sl, 0, hm, s, li, nullptr, 0, 0, cinfo);
        if (FAST && aborted) return;
      }
    }
    {  // 4a: membership change input (rg_config_change)
      const uint32_t v = in_cc;
      if (v && (v & 0xFFu) == s) handle_propose(1, (uint32_t)(P().tick % P().nslab), 0, 0, s, nullptr, nullptr, 0, v >> 8, 0);
    }
    if (in_rd) handle_read_index(my_id(), in_rd);  // 4b: ReadIndex input (rg_read_index)
    RG_STAMP(3);
    if constexpr (LEAN) {
      // the fields only the end of the step reads, loaded here (after a compiler barrier, so their
      // loads are not hoisted to the start of the step and their registers are not held through it)
#if defined(__HIP_DEVICE_COMPILE__) || defined(__GNUC__)
      asm volatile("" ::: "memory");
#endif
      const uint64_t n = P().nrep;
      const uint64_t* a = P().s64 + q;
      processed = processed_start = a[S_PROCESSED * n];
      cc_hi = a[S_CC_HI * n];
      applied = a[S_APPLIED * n];
      snap_index = a[S_SNAP_INDEX * n];
    }
    // GetUpdate.CommittedEntries = (processed, committed], then commitUpdate; applied follows unless
    // the state machine reports it (rg_notify_applied); snapshot + compaction on applied
    // the rsm applies the ConfigChange entries it is handed (none past cc_hi)
    for (uint64_t i = umax64(processed_start, restored_at) + 1; i <= umin64(committed, cc_hi); ++i) {
      const uint64_t w = *tr_at(i);
      if ((w & TYPE_BIT) && word_len(w)) {
        if constexpr (FAST) {  // applying a membership change: the full step's
          abort_();
          return;
        } else {
          apply_config_change(word_len(w));
        }
      }
    }
    processed = committed;
    const bool apv = !P().AF && applied != processed;  // applied moves (the in-place store)
    if (!P().AF) applied = processed;
    if (P().SE && applied >= snap_index && applied - snap_index >= P().SE) {
      snap_index = applied;
      snap_term = term_at(applied);
      snap_members = members;
      took = true;
      const uint64_t c = snap_index > P().CO ? snap_index - P().CO : 0;
      if (c > marker) {
        marker_term = term_at(c);
        marker = c;
      }
    }
    const bool cbv = cap_base != marker_start;
    cap_base = marker_start;
    RG_STAMP(4);
    store(apv, cbv);
    RG_STAMP(5);
#if defined(RG_CTL_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
    if (P().prof)
      for (int k = 0; k < 12; ++k) P().prof[(uint64_t)k * P().nrep + q] = stamps[k];
#endif
  }

  // The step's results, written in place. The full step writes every field. The fast step writes only
  // the fields a fast branch can change, each only when it may have changed this step (apv / cbv:
  // applied and cap_base moved): term, vote, role, the election timer's bound and RNG, the vote masks,
  // the error word, the membership, a pending ConfigChange and cc_hi change only on branches that
  // leave the fast path, and a follower's remotes, heartbeat timer and active mask not at all. In steady
  // state a follower writes its log end, commit and stream rows, a leader those and its remotes.
  RG_FN void store(bool apv, bool cbv) {
    const uint64_t n = P().nrep;
    uint64_t* a = P().s64 + q;
    uint32_t* b = P().s32 + q;
    const bool lmv = last != last_start, mmv = marker != marker_start;
    // the persistence feed (rg_persist_collect): entries written (wlo), or whether the hard state changed
    bool hs;
    if constexpr (FAST) {
      constexpr bool LD = ROLE == (int)LEADER;
      if (RGX(!LD && ldv)) a[S_LEADER * n] = leader;
      if (RGX(cmv)) a[S_COMMITTED * n] = committed;
      if (RGX(processed != processed_start)) a[S_PROCESSED * n] = processed;
      if (RGX(apv)) a[S_APPLIED * n] = applied;
      if (RGX(lmv)) {
        a[S_LAST * n] = last;
        b[S_HW * n] = hw;  // S_LPG / S_APG: pool_kernel (after this launch)
      }
      if (RGX(mmv)) {
        a[S_MARKER * n] = marker;
        a[S_MARKER_TERM * n] = marker_term;
      }
      if (RGX(took)) {
        a[S_SNAP_INDEX * n] = snap_index;
        a[S_SNAP_TERM * n] = snap_term;
        b[S_SNAP_MEMBERS * n] = snap_members;
      }
      if (RGX(cbv)) a[S_CAP_BASE * n] = cap_base;
      // compaction moved the marker: the stream below entry marker + 1 is released by the next step,
      // once this step's bulk kernel has stored that entry's position
      if (RGX(lmv || mmv)) a[S_LAST_TERM * n] = last > marker ? (lt_i == last ? lt_v : *tr_at(last) & TERM_MASK) : marker_term;
      if (RGX2(LD || etick != etick0)) b[S_ETICK * n] = etick;
      if (RGX2(drops != drops0)) b[S_DROPS * n] = drops;
      if (RGX(nlpg_ != lpg_)) b[S_NLPG * n] = nlpg_;  // else S_NLPG = S_LPG already (pool_kernel's last store)
      if constexpr (LD) {
        b[S_HTICK * n] = htick;
        b[S_ACTIVE * n] = active;
        sfor<0, R>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          P().rem[(0 * R + j) * n + q] = rm[j];
          P().rem[(1 * R + j) * n + q] = rn[j];
          P().rst[j * n + q] = (uint8_t)rt[j];
        });
      }
      // term and vote do not change on the fast path
      hs = cmv || lmv || mmv || took;
    } else {
      hs = P().feed && (a[S_TERM * n] != term || a[S_VOTE * n] != vote || a[S_COMMITTED * n] != committed ||
                        lmv || mmv || a[S_SNAP_INDEX * n] != snap_index);
      a[S_TERM * n] = term; a[S_VOTE * n] = vote; a[S_LEADER * n] = leader; a[S_COMMITTED * n] = committed;
      a[S_APPLIED * n] = applied; a[S_LAST * n] = last; a[S_MARKER * n] = marker; a[S_MARKER_TERM * n] = marker_term;
      a[S_SNAP_INDEX * n] = snap_index; a[S_SNAP_TERM * n] = snap_term; a[S_CAP_BASE * n] = cap_base;
      a[S_PROCESSED * n] = processed; a[S_CC_HI * n] = cc_hi;
      a[S_LAST_TERM * n] = last > marker ? (lt_i == last ? lt_v : *tr_at(last) & TERM_MASK) : marker_term;
      b[S_ROLE * n] = role; b[S_ETICK * n] = etick; b[S_HTICK * n] = htick; b[S_RAND_TO * n] = rand_to;
      b[S_RNG_CTR * n] = rng_ctr; b[S_GRANTED * n] = granted; b[S_RESPONDED * n] = responded;
      b[S_ACTIVE * n] = active; b[S_ERR * n] = err; b[S_DROPS * n] = drops;
      b[S_MEMBERS * n] = members; b[S_SNAP_MEMBERS * n] = snap_members; b[S_CC_PENDING * n] = cc_pending;
      b[S_HW * n] = hw;
      b[S_NLPG * n] = nlpg_;
      sfor<0, R>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        P().rem[(0 * R + j) * n + q] = rm[j];
        P().rem[(1 * R + j) * n + q] = rn[j];
        if constexpr (RS_REG) P().rem[(2 * R + j) * n + q] = rs[j];
        P().rst[j * n + q] = (uint8_t)rt[j];
      });
    }
    sfor<0, R>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      P().cnt_out[((uint64_t)RG_S_SEND * R + j) * P().G + g] = get8(oc, j) | (get8(ocls, j) << 8);
    });
    P().jcnt[q] = nj;
    // a restore moved processed to restored_at > processed_start, and commits only grow after it
    if (P().feed)
      P().feed[q] = feed_word(processed, umax64(processed_start, restored_at), last, wlo, wlo != ~0ull || hs,
                              restored_at != 0, took);
  }
#undef RG_GET
#undef RG_SET
};


}  // namespace rg
