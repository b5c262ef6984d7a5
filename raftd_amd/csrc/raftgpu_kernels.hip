// raftgpu_kernels.hip — the MI355X tick kernel: one wavefront steps one Raft replica.
//
// Restates dragonboat v4 internal/raft (raft.go Handle / handleReplicateMessage / tryCommit /
// handleNodeRequestVote / handleCandidateRequestVoteResp / leaderTick / nonLeaderTick,
// logentry.go matchTerm / tryAppend / getConflictIndex / commitTo, remote.go) as specified in
// DESIGN.md §1 — the same contract as oracle/oracle.c, written independently for the GPU.
//
// Execution model (gfx950, wave64):
//  * control is wave-uniform: the replica's scalars live in SGPRs (loaded with s_load from the
//    read-only previous-tick state), branches are scalar;
//  * lane r (< R) holds remote r's {match, next, rsnap, rstate}: reset, quorum counting and the
//    commit order statistic are lane-parallel, single remotes are read with v_readlane;
//  * entry work is lane-parallel: lane e owns entry e of a Replicate / proposal batch (term
//    compare + ballot for the conflict index, term-ring writes), and payload bytes move 16 B
//    per lane, P/16 lanes per entry, with CRC-32 from slice-by-16 tables in LDS combined across
//    the entry's lanes by a shuffle tree of shift tables.
//  * a follower copies payload bytes straight out of the sender's ring (no staging copy);
//    DESIGN.md §2 explains the two payload banks that make this race-free inside one launch.
#include "raftgpu_internal.h"

namespace rg {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ULL;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return z;
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t l) {
  uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
  uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t shfl32(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src, 64); }
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
  uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }

// Order the wave's own earlier global stores before its later loads of the same lines by
// other lanes (same CU: a workgroup-scope fence is a vmcnt drain, no cache maintenance).
__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup"); }

// ------------------------------------------------------------------ CRC-32 in LDS
struct Crc {
  const uint32_t* T;  // LDS [16][256]
  const uint32_t* S;  // LDS [lg][4][256]
  __device__ __forceinline__ uint32_t raw16(uint4 v) const {
    uint32_t r = 0;
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) r ^= T[(15 - (4 * q + j)) * 256 + ((d[q] >> (8 * j)) & 0xFF)];
    return r;
  }
  __device__ __forceinline__ uint32_t shift(uint32_t v, int lvl) const {
    const uint32_t* s = S + lvl * 1024;
    return s[v & 0xFF] ^ s[256 + ((v >> 8) & 0xFF)] ^ s[512 + ((v >> 16) & 0xFF)] ^ s[768 + (v >> 24)];
  }
};

// ------------------------------------------------------------------ one replica's step
enum SrcKind : int { SRC_NONE = 0, SRC_RING = 1, SRC_SLAB = 2 };

struct Step {
  const TickParams& p;
  Crc crc;
  uint32_t rid, g, s, lane;
  // uniform replica state
  uint64_t term, vote, leader, committed, applied, last, marker, marker_term, snap_index, snap_term, cap_base;
  uint32_t role, etick, htick, rand_to, rng_ctr, granted, responded, active, err, drops;
  // remote r in lane r
  uint64_t rmatch, rnext, rsnap;
  uint32_t rstate;
  // step-local
  uint64_t last_start, sent_hi, rw_lo, rw_hi, marker_start;
  uint64_t oc;  // enqueued count per destination, 8 bits each
  uint64_t em;  // emissions per destination (incl. lost), 8 bits each

  __device__ __forceinline__ Step(const TickParams& pp, Crc c, uint32_t r) : p(pp), crc(c), rid(r) {
    lane = lane_id();
    g = rid / p.R;
    s = rid - g * p.R;
    const RepState& st = p.st_in[rid];
    term = st.term; vote = st.vote; leader = st.leader; committed = st.committed; applied = st.applied;
    last = st.last; marker = st.marker; marker_term = st.marker_term; snap_index = st.snap_index;
    snap_term = st.snap_term; cap_base = st.cap_base;
    role = st.role; etick = st.etick; htick = st.htick; rand_to = st.rand_to; rng_ctr = st.rng_ctr;
    granted = st.granted; responded = st.responded; active = st.active; err = st.err; drops = st.drops;
    uint32_t lr = lane < MAX_R ? lane : 0;
    rmatch = st.match[lr]; rnext = st.next[lr]; rsnap = st.rsnap[lr]; rstate = st.rstate[lr];
    last_start = last; sent_hi = 0; rw_lo = ~0ull; rw_hi = 0; marker_start = marker;
    oc = 0; em = 0;
  }

  __device__ __forceinline__ uint32_t quorum() const { return p.R / 2 + 1; }
  __device__ __forceinline__ uint32_t my_id() const { return s + 1; }

  // ---- remotes (lane-resident)
  __device__ __forceinline__ uint64_t M(uint32_t f) const { return rl64(rmatch, f); }
  __device__ __forceinline__ uint64_t N(uint32_t f) const { return rl64(rnext, f); }
  __device__ __forceinline__ uint64_t SN(uint32_t f) const { return rl64(rsnap, f); }
  __device__ __forceinline__ uint32_t ST(uint32_t f) const { return rl(rstate, f); }
  __device__ __forceinline__ void setM(uint32_t f, uint64_t v) { rmatch = lane == f ? v : rmatch; }
  __device__ __forceinline__ void setN(uint32_t f, uint64_t v) { rnext = lane == f ? v : rnext; }
  __device__ __forceinline__ void setSN(uint32_t f, uint64_t v) { rsnap = lane == f ? v : rsnap; }
  __device__ __forceinline__ void setST(uint32_t f, uint32_t v) { rstate = lane == f ? v : rstate; }

  // ---- log (entryLog)
  __device__ __forceinline__ uint64_t* ring_ptr(uint64_t i) const {
    return p.term_ring + (uint64_t)rid * p.L + (i & (p.L - 1));
  }
  __device__ __forceinline__ uint64_t term_at(uint64_t i) const {
    if (i == marker) return marker_term;
    if (i > marker && i <= last) return rfl64(*ring_ptr(i)) & TERM_MASK;
    return 0;
  }
  __device__ __forceinline__ uint64_t last_term() const { return term_at(last); }

  __device__ __forceinline__ void commit_to(uint64_t i) {
    if (i <= committed) return;
    if (i > last) {
      err |= ERR_BEYOND;
      return;
    }
    committed = i;
  }

  // ---- transport
  __device__ __forceinline__ uint32_t get8(uint64_t packed, uint32_t d) const {
    return (uint32_t)(packed >> (8 * d)) & 0xFF;
  }
  __device__ __forceinline__ bool lost(uint32_t dst, uint32_t n) const {
    if (p.isolate && (p.isolate[rid] || p.isolate[g * p.R + dst])) return true;
    if (p.drop_ppm) {
      uint64_t h = mix64(p.seed ^ mix64((p.tick << 40) ^ ((uint64_t)rid << 8) ^ dst) ^ (uint64_t)(n + 1));
      if (h % 1000000ull < p.drop_ppm) return true;
    }
    return false;
  }
  // raft.send + enqueue into the outbox slot. Returns the slot k, or -1 if the message was lost.
  __device__ __forceinline__ int send(uint32_t type, uint32_t to, uint64_t mterm, uint32_t reject, uint32_t nent,
                                      uint64_t log_term, uint64_t log_index, uint64_t commit, uint64_t hint,
                                      uint64_t hint_high, uint32_t src_a, uint32_t src_b) {
    uint32_t dst = to - 1;
    if (type != M_PROPOSE && type != M_REQUEST_VOTE) mterm = term;
    uint32_t n = get8(em, dst);
    em += 1ull << (8 * dst);
    uint32_t k = get8(oc, dst);
    if (lost(dst, n) || k >= p.K) {
      drops++;
      return -1;
    }
    oc += 1ull << (8 * dst);
    MsgHdr* h = p.hdr_out + ((uint64_t)rid * p.R + dst) * p.K + k;
    uint64_t w0 = (uint64_t)type | ((uint64_t)my_id() << 8) | ((uint64_t)to << 16) | ((uint64_t)reject << 24) |
                  ((uint64_t)nent << 32);
    uint64_t w7 = (uint64_t)src_a | ((uint64_t)src_b << 32);
    // lanes 0..7 each store one 8-byte word of the 64-byte slot
    uint64_t v = w0;
    v = lane == 1 ? mterm : v;
    v = lane == 2 ? log_term : v;
    v = lane == 3 ? log_index : v;
    v = lane == 4 ? commit : v;
    v = lane == 5 ? hint : v;
    v = lane == 6 ? hint_high : v;
    v = lane == 7 ? w7 : v;
    if (lane < 8) reinterpret_cast<uint64_t*>(h)[lane] = v;
    return (int)k;
  }
  __device__ __forceinline__ int send_simple(uint32_t type, uint32_t to, uint32_t reject = 0, uint64_t log_index = 0,
                                             uint64_t hint = 0, uint64_t hint_high = 0) {
    return send(type, to, 0, reject, 0, 0, log_index, 0, hint, hint_high, 0, 0);
  }

  // ---- role transitions (A.5)
  __device__ __forceinline__ void reset(uint64_t t) {
    if (t != term) {
      term = t;
      vote = 0;
    }
    leader = 0;
    granted = responded = 0;
    etick = htick = 0;
    rng_ctr++;
    uint64_t key = ((uint64_t)g << 32) | ((uint64_t)s << 24) | (uint64_t)(rng_ctr & 0xFFFFFF);
    rand_to = p.ET + (uint32_t)(mix64(p.seed ^ mix64(key)) % p.ET);
    rmatch = lane == s ? last : 0;
    rnext = last + 1;
    rsnap = 0;
    rstate = RETRY;
    active = 0;
  }
  __device__ __forceinline__ void become_follower(uint64_t t, uint64_t l) {
    role = FOLLOWER;
    reset(t);
    leader = l;
  }
  __device__ __forceinline__ void become_candidate() {
    role = CANDIDATE;
    reset(term + 1);
    leader = 0;
    vote = my_id();
  }

  // remote.tryUpdate
  __device__ __forceinline__ bool remote_try_update(uint32_t f, uint64_t idx) {
    uint64_t nx = N(f), mt = M(f);
    uint32_t st = ST(f);
    if (nx < idx + 1) setN(f, idx + 1);
    if (mt < idx) {
      if (st == WAIT) setST(f, RETRY);
      setM(f, idx);
      return true;
    }
    return false;
  }

  // raft.tryCommit: q = max{m_i : #{j : m_j >= m_i} >= quorum} = sorted_asc[R - quorum]
  __device__ __forceinline__ bool try_commit() {
    uint32_t cnt = 0;
    for (uint32_t j = 0; j < p.R; ++j) cnt += rl64(rmatch, j) >= rmatch ? 1u : 0u;
    uint64_t cand = (lane < p.R && cnt >= quorum()) ? rmatch : 0;
    uint64_t q = 0;
    for (uint32_t j = 0; j < p.R; ++j) q = umax64(q, rl64(cand, j));
    if (q > committed && term_at(q) == term) {
      committed = q;
      return true;
    }
    return false;
  }

  // ---- entry writes (term ring + banks, payload copy + CRC, info ring)
  // Lanes e in [e0, n) write entry index base + e with term tv, type_len tlv.
  // src: RING → sender src_rid, payload bank sbv (per lane), same index; SLAB → slab entry e.
  __device__ void write_entries(uint64_t base, uint32_t e0, uint32_t n, uint64_t tv, uint32_t tlv, int src,
                                uint32_t src_rid, uint32_t sbv, const uint8_t* slab) {
    const uint64_t hi_prot = umax64(last_start, sent_hi);
    const bool mine = lane >= e0 && lane < n;
    const uint64_t idx = base + lane;
    const uint32_t L = p.L;
    const uint64_t slot = idx & (L - 1);
    uint32_t tb = 0;
    if (mine) {  // bank choice
      uint64_t* rp = p.term_ring + (uint64_t)rid * L + slot;
      if (idx <= hi_prot) {
        uint32_t cur = (uint32_t)(*rp >> 63);
        bool in_rw = idx >= rw_lo && idx <= rw_hi;
        tb = in_rw ? cur : cur ^ 1u;
      }
      *rp = tv | ((uint64_t)tb << 63);
    }
    // rewritten-hull bookkeeping (uniform)
    uint64_t lo_w = base + e0, hi_w = umin64(base + n - 1, hi_prot);
    if (lo_w <= hi_w) {
      if (rw_lo > rw_hi) {
        rw_lo = lo_w;
        rw_hi = hi_w;
      } else {
        if (hi_w + 1 < rw_lo) {  // gap below the hull: flip its banks so the hull stays exact
          for (uint64_t gi = hi_w + 1; gi < rw_lo; gi += 64) {
            uint64_t i = gi + lane;
            if (i < rw_lo) {
              uint64_t* rp = p.term_ring + (uint64_t)rid * L + (i & (L - 1));
              *rp ^= BANK_BIT;
            }
          }
        }
        rw_lo = umin64(rw_lo, lo_w);
        rw_hi = umax64(rw_hi, hi_w);
      }
    }
    wave_fence();  // term-ring stores visible to this wave's later lookups

    // payload copy + CRC
    uint32_t crcv = 0;
    const uint32_t P = p.P;
    if (P) {
      const uint32_t lg = 31 - __clz(P >> 4);  // log2(chunks per entry)
      const uint32_t nch = 1u << lg;
      const uint32_t epi = 64u >> lg;  // entries per wave pass
      const uint32_t c = lane & (nch - 1), ei = lane >> lg;
      for (uint32_t b = e0; b < n; b += epi) {
        const uint32_t e = b + ei;
        const uint32_t ec = e < 64 ? e : 63;
        const uint32_t tb_e = shfl32(tb, ec), tl_e = shfl32(tlv, ec), sb_e = shfl32(sbv, ec);
        const bool act = e < n && (tl_e & 0xFFFFFFu) == P;
        uint32_t v = 0;
        if (act) {
          const uint64_t di = base + e;
          uint8_t* dptr = p.pay + (((uint64_t)tb_e * p.nrep + rid) * L + (di & (L - 1))) * P + c * 16;
          const uint8_t* sptr;
          if (src == SRC_RING)
            sptr = p.pay + (((uint64_t)sb_e * p.nrep + src_rid) * L + (di & (L - 1))) * P + c * 16;
          else
            sptr = slab + (uint64_t)e * P + c * 16;
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          u32x4 xv = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(sptr));
          uint4 x = make_uint4(xv.x, xv.y, xv.z, xv.w);
          *reinterpret_cast<uint4*>(dptr) = x;
          v = crc.raw16(x);
        }
        for (uint32_t l = 0; l < lg; ++l) {  // combine chunk CRCs: raw(A||B) = Z^|B|(raw A) ^ raw B
          uint32_t d = 1u << l;
          uint32_t partner = (uint32_t)__shfl_down((int)v, d, 64);
          if ((c & ((d << 1) - 1)) == 0) v = crc.shift(v, (int)l) ^ partner;
        }
        // entry b+i's raw CRC sits in lane i*nch; move it to lane b+i
        const bool take = lane >= b && lane < b + epi;
        uint32_t srcl = take ? ((lane - b) << lg) : 0;
        uint32_t got = shfl32(v, (int)srcl);
        if (take) crcv = got;
      }
      crcv = ((tlv & 0xFFFFFFu) == P) ? (p.crc_const ^ crcv) : 0u;
    }
    if (mine) p.info[((uint64_t)tb * p.nrep + rid) * L + slot] = make_uint2(crcv, tlv);
    if (src == SRC_RING) {  // verify against the sender's stored CRC
      bool bad = false;
      if (mine) bad = p.info[((uint64_t)sbv * p.nrep + src_rid) * L + slot].x != crcv;
      if (__ballot(bad)) err |= ERR_CRC;
    }
  }

  // raft.appendEntries (leader side): n entries at term, from slab (or a len-0 no-op)
  __device__ bool append_local(uint32_t n, int slab_id) {
    if (last + n > cap_base + p.L) return false;
    const uint8_t* slab = nullptr;
    uint32_t tl = (uint32_t)ENTRY_APP << 24;
    if (slab_id >= 0 && p.P) {
      slab = p.slabs + (((uint64_t)slab_id * p.G + g) * p.E) * p.P;
      tl |= p.P;
    }
    write_entries(last + 1, 0, n, term, tl, slab ? SRC_SLAB : SRC_NONE, 0, 0, slab);
    last += n;
    remote_try_update(s, last);
    if (p.R == 1) try_commit();
    return true;
  }

  __device__ void become_leader() {
    role = LEADER;
    reset(term);
    leader = my_id();
    if (!append_local(1, -1)) err |= ERR_RING;
  }

  // ---- replication (A.12)
  __device__ void send_replicate(uint32_t to) {
    uint32_t st = ST(to);
    if (st == WAIT || st == SNAPSHOT) return;
    uint64_t next = N(to);
    if (next <= marker) {  // compacted: InstallSnapshot
      if (!(active & (1u << to))) return;
      if (snap_index == 0) {
        err |= ERR_EMPTY_SNAP;
        return;
      }
      setSN(to, snap_index);
      setST(to, SNAPSHOT);
      send(M_INSTALL_SNAPSHOT, to + 1, 0, 0, 0, snap_term, snap_index, 0, 0, 0, 0, 0);
      return;
    }
    uint32_t n = next <= last ? (uint32_t)umin64(p.E, last - next + 1) : 0;
    uint64_t lt = term_at(next - 1);
    if (n > 0) {  // remote.progress
      if (st == REPLICATE) setN(to, next + n - 1 + 1);
      else if (st == RETRY) setST(to, WAIT);
    }
    int k = send(M_REPLICATE, to + 1, 0, 0, n, lt, next - 1, committed, 0, 0, 0, 0);
    if (k >= 0 && n > 0) {
      if (lane < n) {
        uint64_t* mt = p.mt_out + ((((uint64_t)rid * p.R + to) * p.K + (uint32_t)k) * p.E) + lane;
        *mt = *ring_ptr(next + lane);  // term | bank
      }
      sent_hi = umax64(sent_hi, next + n - 1);
    }
  }
  __device__ void broadcast_replicate() {
    for (uint32_t i = 0; i < p.R; ++i)
      if (i != s) send_replicate(i);
  }
  __device__ void broadcast_heartbeat() {
    for (uint32_t i = 0; i < p.R; ++i) {
      if (i == s) continue;
      send(M_HEARTBEAT, i + 1, 0, 0, 0, 0, 0, umin64(M(i), committed), 0, 0, 0, 0);
    }
  }

  // ---- follower side (A.9)
  __device__ void handle_replicate(const MsgHdr& h, uint32_t from, uint32_t src_slot, uint32_t k) {
    const uint32_t src_rid = g * p.R + src_slot;
    const uint64_t li = h.log_index;
    if (li < committed) {
      send_simple(M_REPLICATE_RESP, from, 0, committed);
      return;
    }
    const uint32_t n = (uint32_t)(h.w0 >> 32);
    if (term_at(li) == h.log_term) {
      // getConflictIndex: lane e compares entry li+1+e
      uint64_t mtv = 0;
      if (lane < n) mtv = p.mt_in[((((uint64_t)src_rid * p.R + s) * p.K + k) * p.E) + lane];
      const uint64_t idx = li + 1 + lane;
      uint64_t mine = 0;
      if (lane < n) {
        if (idx == marker) mine = marker_term;
        else if (idx > marker && idx <= last) mine = *ring_ptr(idx) & TERM_MASK;
      }
      const uint64_t bal = __ballot(lane < n && mine != (mtv & TERM_MASK));
      const uint64_t last_new = li + n;
      if (bal) {
        const uint32_t k0 = (uint32_t)__builtin_ctzll(bal);
        const uint64_t ci = li + 1 + k0;
        if (ci > committed && last_new > cap_base + p.L) {
          drops++;  // capacity rule: dropped, no reply
          return;
        }
        if (ci <= committed) {
          err |= ERR_CONFLICT;
        } else {
          uint32_t sb = (uint32_t)(mtv >> 63);
          uint32_t tl = 0;
          if (lane >= k0 && lane < n)
            tl = p.info[((uint64_t)sb * p.nrep + src_rid) * p.L + (idx & (p.L - 1))].y;
          write_entries(li + 1, k0, n, mtv & TERM_MASK, tl, SRC_RING, src_rid, sb, nullptr);
          last = last_new;
        }
      }
      commit_to(umin64(last_new, h.commit));
      send_simple(M_REPLICATE_RESP, from, 0, last_new);
    } else {
      send_simple(M_REPLICATE_RESP, from, 1, li, last);
    }
  }

  __device__ void handle_install_snapshot(const MsgHdr& h, uint32_t from) {
    const uint64_t si = h.log_index, stt = h.log_term;
    uint64_t li;
    if (si <= committed) {
      li = committed;
    } else if (term_at(si) == stt) {
      commit_to(si);
      li = committed;
    } else {  // restore
      marker = last = committed = snap_index = si;
      marker_term = snap_term = stt;
      li = last;
    }
    send_simple(M_REPLICATE_RESP, from, 0, li);
  }

  // ---- elections (A.7, A.8)
  __device__ void campaign() {
    become_candidate();
    responded |= 1u << s;
    granted |= 1u << s;
    if (p.R == 1) {
      become_leader();
      return;
    }
    uint64_t lt = last_term();
    for (uint32_t i = 0; i < p.R; ++i) {
      if (i == s) continue;
      send(M_REQUEST_VOTE, i + 1, term, 0, 0, lt, last, 0, 0, 0, 0, 0);
    }
  }
  __device__ void handle_node_election() {
    if (role == LEADER) return;
    if (committed > applied) return;  // hasConfigChangeToApply
    campaign();
  }
  __device__ void handle_request_vote(const MsgHdr& h, uint32_t from) {
    bool can = vote == 0 || vote == from;
    uint64_t lt = last_term();
    bool utd = h.log_term > lt || (h.log_term == lt && h.log_index >= last);
    uint32_t rej = 1;
    if (can && utd) {
      etick = 0;
      vote = from;
      rej = 0;
    }
    send_simple(M_REQUEST_VOTE_RESP, from, rej);
  }
  __device__ void candidate_vote_resp(uint32_t from, uint32_t reject) {
    uint32_t bit = 1u << (from - 1);
    if (!(responded & bit)) {
      responded |= bit;
      if (!reject) granted |= bit;
    }
    uint32_t gr = __builtin_popcount(granted), tot = __builtin_popcount(responded);
    if (gr == quorum()) {
      become_leader();
      broadcast_replicate();
    } else if (tot - gr == quorum()) {
      become_follower(term, 0);
    }
  }

  // ---- leader responses (A.10, A.11)
  __device__ void leader_replicate_resp(const MsgHdr& h, uint32_t from) {
    const uint32_t f = from - 1;
    active |= 1u << f;
    const uint32_t reject = (uint32_t)(h.w0 >> 24) & 0xFF;
    if (!reject) {
      uint32_t st0 = ST(f);
      bool paused = st0 == WAIT || st0 == SNAPSHOT;
      if (remote_try_update(f, h.log_index)) {
        uint32_t st = ST(f);
        if (st == RETRY) {  // respondedTo → becomeReplicate
          setN(f, M(f) + 1);
          setSN(f, 0);
          setST(f, REPLICATE);
        } else if (st == SNAPSHOT && M(f) >= SN(f)) {  // becomeRetry from Snapshot
          setN(f, umax64(M(f) + 1, SN(f) + 1));
          setSN(f, 0);
          setST(f, RETRY);
        }
        if (try_commit()) broadcast_replicate();
        else if (paused) send_replicate(f);
      }
    } else {  // remote.decreaseTo
      const uint64_t rej = h.log_index, hint = h.hint;
      const uint32_t st = ST(f);
      bool ok;
      if (st == REPLICATE) {
        if (rej <= M(f)) ok = false;
        else {
          setN(f, M(f) + 1);
          ok = true;
        }
      } else if (N(f) - 1 != rej) {
        ok = false;
      } else {
        if (st == WAIT) setST(f, RETRY);
        setN(f, umax64(1, umin64(rej, hint + 1)));
        ok = true;
      }
      if (ok) {
        if (ST(f) == REPLICATE) {  // enterRetryState → becomeRetry
          setN(f, M(f) + 1);
          setSN(f, 0);
          setST(f, RETRY);
        }
        send_replicate(f);
      }
    }
  }
  __device__ void leader_heartbeat_resp(uint32_t from) {
    const uint32_t f = from - 1;
    active |= 1u << f;
    if (ST(f) == WAIT) setST(f, RETRY);
    if (M(f) < last) send_replicate(f);
  }
  __device__ void check_quorum() {
    uint32_t c = 1 + __builtin_popcount(active & ~(1u << s));
    active = 0;
    if (c < quorum()) become_follower(term, 0);
  }

  // ---- proposals
  __device__ void handle_propose(uint32_t nent, uint32_t slab_id, uint32_t hop) {
    if (role == LEADER) {
      if (!append_local(nent, (int)slab_id)) {
        drops++;
        return;
      }
      broadcast_replicate();
    } else if (role == FOLLOWER && leader != 0 && hop == 0) {
      send(M_PROPOSE, (uint32_t)leader, 0, 0, nent, 0, 0, 0, 0, 0, slab_id, hop + 1);
    } else {
      drops++;
    }
  }

  // ---- timers (A.6)
  __device__ void tick() {
    if (role == LEADER) {
      etick++;
      if (etick >= p.ET) {
        etick = 0;
        if (p.CQ) check_quorum();
      }
      htick++;
      if (htick >= p.HT) {
        htick = 0;
        if (role == LEADER) broadcast_heartbeat();
      }
    } else {
      etick++;
      if (etick >= rand_to) {
        etick = 0;
        handle_node_election();
      }
    }
  }

  // ---- Handle (A.3) for a message from another replica
  __device__ void handle(const MsgHdr& h, uint32_t src_slot, uint32_t k) {
    const uint32_t type = (uint32_t)(h.w0 & 0xFF);
    const uint32_t from = (uint32_t)(h.w0 >> 8) & 0xFF;
    const uint64_t mterm = h.term;
    const bool leader_msg = type == M_REPLICATE || type == M_INSTALL_SNAPSHOT || type == M_HEARTBEAT;
    if (mterm != 0 && mterm != term) {
      if (type == M_REQUEST_VOTE && p.CQ && mterm > term && h.hint != from && leader != 0 && etick < p.ET) return;
      if (mterm > term) {
        become_follower(mterm, leader_msg ? from : 0);
      } else {
        if (p.CQ && leader_msg) send_simple(M_NOOP, from);
        return;
      }
    }
    switch (type) {
      case M_PROPOSE:
        handle_propose((uint32_t)(h.w0 >> 32), (uint32_t)h.w7, (uint32_t)(h.w7 >> 32));
        break;
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
          handle_replicate(h, from, src_slot, k);
        } else if (type == M_HEARTBEAT) {
          commit_to(h.commit);
          send_simple(M_HEARTBEAT_RESP, from, 0, 0, h.hint, h.hint_high);
        } else {
          handle_install_snapshot(h, from);
        }
        break;
      case M_REPLICATE_RESP:
        if (role == LEADER) leader_replicate_resp(h, from);
        break;
      case M_HEARTBEAT_RESP:
        if (role == LEADER) leader_heartbeat_resp(from);
        break;
      case M_REQUEST_VOTE:
        handle_request_vote(h, from);
        break;
      case M_REQUEST_VOTE_RESP:
        if (role == CANDIDATE) candidate_vote_resp(from, (uint32_t)(h.w0 >> 24) & 0xFF);
        break;
      default:
        break;
    }
  }

  // ---- the whole step
  __device__ void run() {
    const uint32_t R = p.R;
    for (uint32_t src = 0; src < R; ++src) {
      if (src == s) continue;
      const uint32_t srid = g * R + src;
      const uint32_t cnt = p.cnt_in[(uint64_t)srid * R + s];
      for (uint32_t k = 0; k < cnt; ++k) {
        const MsgHdr h = p.hdr_in[((uint64_t)srid * R + s) * p.K + k];
        handle(h, src, k);
      }
    }
    if (p.campaign && p.campaign[rid]) handle_node_election();
    if (!(p.flags & 1u)) tick();
    if (p.prop_target && p.prop_target[g] == s) {
      uint32_t n = p.prop_count[g];
      if (n > 0) handle_propose(n, (uint32_t)(p.tick % p.nslab), 0);
    }
    // apply, snapshot, compaction
    applied = committed;
    if (p.SE && applied - snap_index >= p.SE) {
      snap_index = applied;
      snap_term = term_at(applied);
      uint64_t c = snap_index > p.CO ? snap_index - p.CO : 0;
      if (c > marker) {
        marker_term = term_at(c);
        marker = c;
      }
    }
    cap_base = marker_start;
    store();
  }

  __device__ void store() {
    RepState& o = p.st_out[rid];
    if (lane == 0) {
      o.term = term; o.vote = vote; o.leader = leader; o.committed = committed; o.applied = applied;
      o.last = last; o.marker = marker; o.marker_term = marker_term; o.snap_index = snap_index;
      o.snap_term = snap_term; o.cap_base = cap_base;
      o.role = role; o.etick = etick; o.htick = htick; o.rand_to = rand_to; o.rng_ctr = rng_ctr;
      o.granted = granted; o.responded = responded; o.active = active; o.err = err; o.drops = drops;
    }
    if (lane < p.R) {
      o.match[lane] = rmatch;
      o.next[lane] = rnext;
      o.rsnap[lane] = rsnap;
      o.rstate[lane] = (uint8_t)rstate;
      p.cnt_out[(uint64_t)rid * p.R + lane] = get8(oc, lane);
    }
  }
};

__global__ void __launch_bounds__(256) tick_kernel(TickParams p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t lgP = p.P ? 31 - __clz(p.P >> 4) : 0;
  const uint32_t words = CRC_T_WORDS + lgP * 1024;
  if (p.P) {
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) lds[i] = p.crc_tab[i];
  }
  __syncthreads();
  Crc crc{lds, lds + CRC_T_WORDS};
  // one replica per wave: a grid-stride loop here makes hipcc keep ~2x the VGPRs live
  const uint32_t rid = rfl(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  if (rid < p.nrep) {
    Step st(p, crc, rid);
    st.run();
  }
}

int tick_lds_bytes(uint32_t P) {
  uint32_t lg = 0;
  if (P) {
    uint32_t nch = P >> 4;
    while ((1u << lg) < nch) ++lg;
    return (int)((CRC_T_WORDS + lg * 1024) * 4);
  }
  return 16;
}

int tick_blocks_per_cu(uint32_t P) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, tick_kernel, 256, tick_lds_bytes(P)) != hipSuccess) n = 4;
  return n > 0 ? n : 1;
}

hipError_t launch_tick(const TickParams& p, hipStream_t s, int grid) {
  hipLaunchKernelGGL(tick_kernel, dim3(grid), dim3(256), tick_lds_bytes(p.P), s, p);
  return hipGetLastError();
}

// ------------------------------------------------------------------ bootstrap (peer.go Launch + bootstrap)
__global__ void bootstrap_kernel(TickParams p) {
  const uint32_t rid = blockIdx.x * blockDim.x + threadIdx.x;
  if (rid >= p.nrep) return;
  const uint32_t R = p.R, g = rid / R, s = rid - g * R;
  RepState st{};
  st.term = 1;  // becomeFollower(1, NoLeader): one reset
  st.rng_ctr = 1;
  uint64_t key = ((uint64_t)g << 32) | ((uint64_t)s << 24) | 1ull;
  st.rand_to = p.ET + (uint32_t)(mix64(p.seed ^ mix64(key)) % p.ET);
  st.last = R;
  st.committed = R;
  for (uint32_t k = 0; k < R; ++k) {  // addNode → setRemote(id, 0, last+1)
    st.next[k] = R + 1;
  }
  p.st_out[rid] = st;
  for (uint32_t i = 1; i <= R; ++i) {
    p.term_ring[(uint64_t)rid * p.L + (i & (p.L - 1))] = 1;  // term 1, bank 0
    p.info[(uint64_t)rid * p.L + (i & (p.L - 1))] = make_uint2(0u, (uint32_t)ENTRY_CONFIG << 24);
  }
  for (uint32_t d = 0; d < R; ++d) p.cnt_out[(uint64_t)rid * R + d] = 0;
}

hipError_t launch_bootstrap(const TickParams& p, hipStream_t s) {
  hipLaunchKernelGGL(bootstrap_kernel, dim3((p.nrep + 255) / 256), dim3(256), 0, s, p);
  return hipGetLastError();
}

// ------------------------------------------------------------------ proposal payload generator
__global__ void fill_slabs_kernel(uint8_t* slabs, uint32_t nslab, uint32_t G, uint32_t E, uint32_t P, uint64_t seed) {
  const uint64_t words_per_entry = P / 8;
  const uint64_t total = (uint64_t)nslab * G * E * words_per_entry;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < total; w += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t ent = w / words_per_entry, wi = w - ent * words_per_entry;
    uint32_t i = (uint32_t)(ent % E);
    uint64_t sg = ent / E;
    uint32_t gg = (uint32_t)(sg % G), sl = (uint32_t)(sg / G);
    uint64_t key = mix64(((uint64_t)sl << 56) ^ ((uint64_t)gg << 16) ^ (uint64_t)i ^ (seed * 0x9E3779B97F4A7C15ULL));
    reinterpret_cast<uint64_t*>(slabs)[w] = mix64(key + (wi + 1) * 0xD1B54A32D192ED03ULL);
  }
}

hipError_t launch_fill_slabs(uint8_t* slabs, uint32_t nslab, uint32_t G, uint32_t E, uint32_t P, uint64_t seed,
                             hipStream_t s) {
  if (!P) return hipSuccess;
  hipLaunchKernelGGL(fill_slabs_kernel, dim3(4096), dim3(256), 0, s, slabs, nslab, G, E, P, seed);
  return hipGetLastError();
}

// ------------------------------------------------------------------ Σ_g max_s committed
__global__ void sum_committed_kernel(const RepState* st, uint32_t G, uint32_t R, unsigned long long* out) {
  uint64_t acc = 0;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) {
    uint64_t m = 0;
    for (uint32_t k = 0; k < R; ++k) m = umax64(m, st[(uint64_t)g * R + k].committed);
    acc += m;
  }
  for (int off = 32; off > 0; off >>= 1) {
    uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)acc, off, 64);
    uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(acc >> 32), off, 64);
    acc += ((uint64_t)hi << 32) | lo;
  }
  if (lane_id() == 0) atomicAdd(out, (unsigned long long)acc);
}

hipError_t launch_sum_committed(const RepState* st, uint32_t G, uint32_t R, unsigned long long* out, hipStream_t s) {
  hipLaunchKernelGGL(sum_committed_kernel, dim3(256), dim3(256), 0, s, st, G, R, out);
  return hipGetLastError();
}

// ------------------------------------------------------------------ last-tick traffic accounting
// out6: leaders, msgs, repl_entries, appended, leader_appended, (unused)
__global__ void traffic_kernel(TickParams p, const RepState* st_prev, unsigned long long* out6) {
  uint64_t v[5] = {0, 0, 0, 0, 0};
  for (uint32_t rid = blockIdx.x * blockDim.x + threadIdx.x; rid < p.nrep; rid += gridDim.x * blockDim.x) {
    const RepState& cur = p.st_in[rid];
    const bool ld = cur.role == LEADER;
    v[0] += ld;
    for (uint32_t d = 0; d < p.R; ++d) {
      const uint32_t n = p.cnt_in[(uint64_t)rid * p.R + d];
      v[1] += n;
      for (uint32_t k = 0; k < n; ++k) {
        const MsgHdr& h = p.hdr_in[((uint64_t)rid * p.R + d) * p.K + k];
        if ((h.w0 & 0xFF) == M_REPLICATE) v[2] += h.w0 >> 32;
      }
    }
    const uint64_t app = cur.last > st_prev[rid].last ? cur.last - st_prev[rid].last : 0;
    v[3] += app;
    if (ld) v[4] += app;
  }
  for (int i = 0; i < 5; ++i) {
    uint64_t a = v[i];
    for (int off = 32; off > 0; off >>= 1) {
      uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)a, off, 64);
      uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(a >> 32), off, 64);
      a += ((uint64_t)hi << 32) | lo;
    }
    if (lane_id() == 0 && a) atomicAdd(out6 + i, (unsigned long long)a);
  }
}

hipError_t launch_traffic(const TickParams& p, const RepState* st_prev, unsigned long long* out6, hipStream_t s) {
  hipLaunchKernelGGL(traffic_kernel, dim3(512), dim3(256), 0, s, p, st_prev, out6);
  return hipGetLastError();
}

}  // namespace rg
