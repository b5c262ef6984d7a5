// raftgpu_kernels.hip — the MI355X Raft tick: a control kernel (all Raft logic, one lane per
// replica) followed by a bulk kernel (entry payload copy + CRC-32, one wavefront per replica).
//
// Restates dragonboat v4 internal/raft (raft.go Handle / handleReplicateMessage / tryCommit /
// handleNodeRequestVote / handleCandidateRequestVoteResp / leaderTick / nonLeaderTick,
// logentry.go matchTerm / tryAppend / getConflictIndex / commitTo, remote.go) as specified in
// DESIGN.md §1 — the same contract as oracle/oracle.c, written independently for the GPU.
//
// control_kernel<R>: lane q steps replica q (slot-major numbering, see raftgpu_internal.h). Its
//   state, the message slots and the term ring are structure-of-arrays indexed by q or by group,
//   so each per-lane access is a coalesced wave access. It touches only metadata: terms, indices,
//   message headers, inline entry terms. Every log append becomes a job record (index range,
//   source, per-entry bank / payload / type bits) for the bulk kernel.
// bulk_kernel: for each job, lanes move payload 16 B per lane (P/16 lanes per entry, 8 chunks in
//   flight per lane), write the destination ring, and compute CRC-32 per entry from slice-by-16
//   LDS tables, combined across the entry's lanes by a shuffle tree of shift tables; followers
//   check the result against the sender's stored CRC. Payloads are read straight from the
//   sender's ring (no staging copy); DESIGN.md §2 explains the two payload banks that keep the
//   same-launch reads and rewrites disjoint.
#include <algorithm>

#include "raftgpu_control.h"

namespace rg {

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

#ifndef RG_CTL_MINWAVES
#define RG_CTL_MINWAVES 1
#endif
#ifndef RG_CTL_BLOCK
#define RG_CTL_BLOCK 64  // lanes per control workgroup: one wave, so a SIMD starts the next wave as soon as
                         // its last one ends (r02 A/B vs 256: control 0.122 -> 0.118 ms at 64K x 3, C2 0.043 -> 0.041)
#endif
// The parameter block comes by pointer from a device slot the host filled with a stream-ordered
// copy (DESIGN.md §3 "The control-kernel fault"); Ctl copies it (scalar loads, uniform address).
template <int R>
__global__ void __launch_bounds__(RG_CTL_BLOCK, RG_CTL_MINWAVES) control_kernel(const TickParams* __restrict__ pp) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  const TickParams p = *pp;
  if (q >= p.nrep) return;
#ifdef RG_CTL_PROFILE
  const uint32_t t0 = (uint32_t)__builtin_amdgcn_s_memtime();
  Ctl<R> c(p, q);
  c.stamps[0] = t0;
#else
  Ctl<R> c(p, q);
#endif
  c.run();
}

hipError_t launch_control(const TickParams* p, uint32_t R, uint32_t nrep, hipStream_t s) {
  dim3 grid((nrep + RG_CTL_BLOCK - 1) / RG_CTL_BLOCK), block(RG_CTL_BLOCK);
  switch (R) {
    case 1: hipLaunchKernelGGL(control_kernel<1>, grid, block, 0, s, p); break;
    case 2: hipLaunchKernelGGL(control_kernel<2>, grid, block, 0, s, p); break;
    case 3: hipLaunchKernelGGL(control_kernel<3>, grid, block, 0, s, p); break;
    case 4: hipLaunchKernelGGL(control_kernel<4>, grid, block, 0, s, p); break;
    case 5: hipLaunchKernelGGL(control_kernel<5>, grid, block, 0, s, p); break;
    case 6: hipLaunchKernelGGL(control_kernel<6>, grid, block, 0, s, p); break;
    case 7: hipLaunchKernelGGL(control_kernel<7>, grid, block, 0, s, p); break;
    case 8: hipLaunchKernelGGL(control_kernel<8>, grid, block, 0, s, p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ================================================================== bulk kernel
struct Crc {
  const uint32_t* T;   // LDS [16][256] byte tables
  const uint32_t* N;   // LDS [16][2][16] nibble tables
  const uint32_t* SH;  // LDS this lane's [8][16] shift table
  // raw CRC contribution of a 16-byte chunk taken as the last 16 bytes of a message
  __device__ __forceinline__ uint32_t raw16(uint4 v) const {
    uint32_t r = 0;
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#ifdef RG_CRC_NIBBLE  // ablation: twice the lookups into conflict-free 16-word tables (VALU-bound: slower)
#pragma unroll
    for (int qd = 0; qd < 4; ++qd)
#pragma unroll
      for (int h = 0; h < 8; ++h) r ^= N[((15 - (4 * qd + (h >> 1))) * 2 + (h & 1)) * 16 + ((d[qd] >> (4 * h)) & 0xF)];
#else
#pragma unroll
    for (int qd = 0; qd < 4; ++qd)
#pragma unroll
      for (int j = 0; j < 4; ++j) r ^= T[(15 - (4 * qd + j)) * 256 + ((d[qd] >> (8 * j)) & 0xFF)];
#endif
    return r;
  }
  // Z^(16·(NCH−1−c))(v): move this lane's chunk contribution to the end of the entry
  __device__ __forceinline__ uint32_t shift(uint32_t v) const {
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r ^= SH[j * 16 + ((v >> (4 * j)) & 0xF)];
    return r;
  }
};

// XOR over the 2^LG lanes of an entry (aligned lane groups); DPP within a row, shuffles across rows
template <int LG>
__device__ __forceinline__ uint32_t xor_lanes(uint32_t v) {
  if constexpr (LG >= 1) v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
  if constexpr (LG >= 2) v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad_perm 2,3,0,1
  if constexpr (LG >= 3) v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  if constexpr (LG >= 4) v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);  // row_mirror
  if constexpr (LG >= 5) v ^= (uint32_t)__shfl_xor((int)v, 16, 64);
  if constexpr (LG >= 6) v ^= (uint32_t)__shfl_xor((int)v, 32, 64);
  return v;
}

#ifndef RG_BULK_U
#define RG_BULK_U 4
#endif
constexpr int BULK_U = RG_BULK_U;  // 16-B chunks in flight per lane

// One copy job, its fields uniform across the wave (SGPRs): n entries from `first`, payloads
// from the sender's ring or a proposal slab into this replica's ring, CRC per entry.
struct Job {
  uint64_t first, dm, sm, hm, tm;
  uint32_t meta, src;
};

__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t l) {
  // readlane returns int: widen through uint32_t, or bit 31 of the low word sign-extends over the high word
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ Job load_job(const BulkParams& p, uint32_t q, uint32_t j) {
  const uint64_t JN = (uint64_t)p.J * p.nrep, jq = (uint64_t)j * p.nrep + q;
  Job jb;
  jb.first = p.job64[J_FIRST * JN + jq];
  jb.dm = p.job64[J_DMASK * JN + jq];
  jb.sm = p.job64[J_SMASK * JN + jq];
  jb.hm = p.job64[J_HMASK * JN + jq];
  jb.tm = p.job64[J_TMASK * JN + jq];
  jb.meta = p.job32[J_META * JN + jq];
  jb.src = p.job32[J_SRC * JN + jq];
  return jb;
}

// ---- software-pipelined payload stream.
// A wave walks a flat sequence of steps over the jobs of its tiles; one step = epi entries of one
// job, 16 B per lane. BULK_U steps are in flight at once in a register ring: slot u is consumed
// (store, CRC, info, verify) and immediately re-issued with the step BULK_U ahead. All cursor
// state is wave-uniform (SGPRs).
struct Cursor {
  uint32_t t, q, qb, g, njl, j, n, kind, src, b;
  uint64_t m, first, dm, sm, hm, tm;
  bool live;
};

struct TileJobs {  // per lane: job count and first job of replica qb + lane
  uint32_t nj;
  Job j0;
};

// Tiles interleave the slots of one block of groups: tile t = (group block t / R, slot t % R), so
// the R replicas of the same groups are walked by neighbouring waves at the same time and the two
// followers' reads of their leader's new entries meet in L2 / Infinity Cache instead of both going
// to HBM (slot-major tiles put them a third of the launch apart). RG_TILE_SLOTMAJOR: ablation.
__device__ __forceinline__ uint32_t bulk_ntiles(const BulkParams& p) {
#ifdef RG_TILE_SLOTMAJOR
  return (p.nrep + p.tile - 1) / p.tile;
#else
  return p.R * ((p.G + p.tile - 1) / p.tile);
#endif
}

__device__ __forceinline__ void load_tile(const BulkParams& p, Cursor& cur, TileJobs& tj) {
  const uint32_t lane = lane_id();
#ifdef RG_TILE_SLOTMAJOR
  cur.qb = cur.t * p.tile;
  const bool valid = lane < p.tile && cur.qb + lane < p.nrep;
#else
  const uint32_t b = cur.t / p.R, s = cur.t - b * p.R, g0 = b * p.tile;
  cur.qb = s * p.G + g0;
  const bool valid = lane < p.tile && g0 + lane < p.G;
#endif
  const uint32_t q = cur.qb + lane;
  tj.nj = valid ? p.jcnt[q] : 0u;
  tj.j0 = Job{};
  if (tj.nj) tj.j0 = load_job(p, q, 0);
  cur.m = __ballot(tj.nj != 0);
  cur.j = 0;
  cur.njl = 0;
}

template <bool WIRE>
__device__ __forceinline__ void set_job(const BulkParams& p, Cursor& cur, const Job& jb) {
  cur.first = jb.first; cur.dm = jb.dm; cur.sm = jb.sm; cur.hm = jb.hm; cur.tm = jb.tm;
  cur.n = jb.meta & 0xFF; cur.b = (jb.meta >> 8) & 0xFF; cur.kind = (jb.meta >> 16) & 0xF; cur.src = jb.src;
  cur.g = WIRE ? (cur.src >> 16) * p.G + cur.q % p.G : cur.q % p.G;  // SRC_SLAB: the proposal's slab row
  cur.src &= cur.kind == SRC_SLAB ? 0xFFFFu : 0xFFFFFFFFu;
  // a malformed job (never produced by control_kernel) is skipped and marks its replica ERR_WIRE
  const bool bad = cur.n > 64 || cur.b > cur.n || (cur.kind == SRC_RING && cur.src >= p.nrep) ||
                   (cur.kind == SRC_SLAB && (cur.src >= p.nslab || cur.g >= (WIRE ? p.nrep : p.G))) ||
                   cur.kind > SRC_WIRE_PROP ||
                   (cur.kind == SRC_WIRE && (!p.wire_mode || cur.n > cur.src ||
                                             cur.sm + (16ull + p.P) * cur.src > p.wire_bytes));
  if (bad) {
#ifdef RG_BOUNDS
    if (lane_id() == 0)
      printf("RG_BOUNDS bulk q=%u job=%u n=%u b=%u kind=%u src=%u sm=%llu wire_bytes=%llu\n", cur.q, cur.j, cur.n,
             cur.b, cur.kind, cur.src, (unsigned long long)cur.sm, (unsigned long long)p.wire_bytes);
#endif
    if (lane_id() == 0) atomicOr(p.crc_err + cur.q, ERR_WIRE);
    cur.n = 0;
    cur.b = 0;
  }
}

// Move the cursor one position: the replica's next job, the tile's next replica, or the next
// tile (whose descriptors arrive in one round trip; that pass issues nothing). A job with no
// entries left to write simply yields an empty pass. Returns false once the wave is done.
template <bool WIRE = false>
__device__ __forceinline__ bool next_job(const BulkParams& p, Cursor& cur, TileJobs& tj, uint32_t stride,
                                         uint32_t ntiles) {
  if (cur.j + 1 < cur.njl) {
    ++cur.j;
    set_job<WIRE>(p, cur, load_job(p, cur.q, cur.j));
  } else if (cur.m) {
    const uint32_t l = rfl((uint32_t)__ffsll((long long)cur.m) - 1);
    cur.m &= cur.m - 1;
    cur.q = cur.qb + l;
    cur.njl = __builtin_amdgcn_readlane(tj.nj, l);
    cur.j = 0;
    Job jb;
    jb.first = rl64(tj.j0.first, l); jb.dm = rl64(tj.j0.dm, l); jb.sm = rl64(tj.j0.sm, l);
    jb.hm = rl64(tj.j0.hm, l); jb.tm = rl64(tj.j0.tm, l);
    jb.meta = __builtin_amdgcn_readlane(tj.j0.meta, l); jb.src = __builtin_amdgcn_readlane(tj.j0.src, l);
    set_job<WIRE>(p, cur, jb);
  } else {
    cur.t += stride;
    if (cur.t >= ntiles) return false;
    load_tile(p, cur, tj);
    cur.b = 0;  // two statements: the chained form kept Cursor in scratch
    cur.n = 0;
  }
  return true;
}

enum : uint32_t { F_ACT = 1, F_WRITER = 2, F_TYPE = 4, F_CHECK = 8 };


// P = 16 << LG bytes per entry: 2^LG lanes per entry (16 B each), 64 >> LG entries per step.
// WIRE: the engine exchanges messages with other ranks (SRC_WIRE jobs, slab rows per replica);
// one-rank engines run the variant without those paths.
template <int LG, bool WIRE>
__global__ void __launch_bounds__(256) bulk_kernel(BulkParams p) {
  constexpr uint32_t NCH = 1u << LG, EPI = 64u >> LG, P = 16u << LG;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  for (uint32_t i = threadIdx.x; i < CRC_T_WORDS + CRC_N_WORDS + NCH * CRC_SH_STRIDE; i += blockDim.x)
    lds[i] = p.crc_tab[i];
  __syncthreads();
  const uint32_t waves = blockDim.x >> 6, lane = lane_id();
  const uint32_t stride = gridDim.x * waves;
  const uint32_t ntiles = bulk_ntiles(p);
  const uint64_t n64 = p.nrep, L = p.L, rows = WIRE ? p.nrep : p.G;
  const uint32_t c = lane & (NCH - 1), ei = lane >> LG;
  const Crc crc{lds, lds + CRC_T_WORDS, lds + CRC_T_WORDS + CRC_N_WORDS + c * CRC_SH_STRIDE};
  Cursor cur{};
  TileJobs tj{};
  cur.t = rfl(blockIdx.x * waves + (threadIdx.x >> 6));
  if (cur.t >= ntiles) return;
  load_tile(p, cur, tj);
  cur.b = 0;  // two statements: the chained form kept Cursor in scratch
  cur.n = 0;
  cur.live = next_job<WIRE>(p, cur, tj, stride, ntiles);
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  // ring slot u: payload chunk, destination (slot | bank << 31), flags, sender's slot CRC
  u32x4 x[BULK_U];
  uint32_t ds[BULK_U], fl[BULK_U], want[BULK_U];
#pragma unroll
  for (int u = 0; u < BULK_U; ++u) {
    x[u] = u32x4{0, 0, 0, 0};
    ds[u] = fl[u] = want[u] = 0;
  }
  // Every slot issues exactly two loads per pass (payload chunk + sender CRC word), redirected to a
  // dummy address when the slot has no work, so the number of memory operations between a load
  // and its use is the same on every path and the compiler's vmcnt waits keep the ring in flight.
  // A pass never spans two jobs (the cursor moves once per pass), so the slots consumed in a pass
  // all belong to the replica `cq` of the previous pass.
  const uint8_t* dummy = reinterpret_cast<const uint8_t*>(p.crc_tab);
  uint32_t vmask = 0, iq = 0;
  do {
    const uint32_t cq = iq;
    iq = cur.q;
    const uint64_t cbase = (uint64_t)cq * L;
#pragma unroll
    for (int u = 0; u < BULK_U; ++u) {
      {  // consume slot u: store, CRC, info, verify (fl = 0 for an empty slot: no stores). A payload
        // slot holds the Cmd zero-padded to P bytes (every writer copies whole slots), so the CRC is
        // the slot CRC; the Cmd's length lives in the term word, not here.
        const bool act = fl[u] & F_ACT;
        const uint64_t di = (uint64_t)(ds[u] >> 31) * n64 * L + cbase + (ds[u] & 0x7FFFFFFFu);
        if (act) {
#ifdef RG_BULK_PLAIN_STORE
          *reinterpret_cast<u32x4*>(p.pay + di * P + c * 16) = x[u];
#else
          __builtin_nontemporal_store(x[u], reinterpret_cast<u32x4*>(p.pay + di * P + c * 16));
#endif
        }
        uint32_t v = 0;
#ifndef RG_BULK_NOCRC
        v = crc.raw16(make_uint4(x[u].x, x[u].y, x[u].z, x[u].w));
#endif
        if constexpr (LG > 0) v = xor_lanes<LG>(crc.shift(v));  // raw(slot) = XOR_c Z^(after c)(raw c)
        if (fl[u] & F_WRITER) {
          const uint32_t cr = act ? (p.crc_const ^ v) : 0u;
          const uint32_t tl = ((fl[u] & F_TYPE) ? (1u << 24) : 0u) | (act ? P : 0u);
          p.info[di] = make_uint2(cr, tl);
          if ((fl[u] & F_CHECK) && want[u] != cr) atomicOr(p.crc_err + cq, ERR_CRC);
        }
      }
      {  // issue the job's next step (or an empty step) into slot u
        const bool step = cur.live && cur.b < cur.n;
        const uint32_t e = cur.b + ei;
        const bool valid = step && e < cur.n;
        const bool act = valid && ((cur.hm >> e) & 1ull);
        const uint32_t slot = (uint32_t)((cur.first + e) & (L - 1));
        const uint32_t db = valid ? (uint32_t)(cur.dm >> e) & 1u : 0u;
        const bool ring = cur.kind == SRC_RING, wire = WIRE && (cur.kind == SRC_WIRE || cur.kind == SRC_WIRE_PROP);
        ds[u] = slot | (db << 31);
        fl[u] = (act ? F_ACT : 0u) | ((valid && c == 0) ? F_WRITER : 0u) | (((cur.tm >> e) & 1ull) ? F_TYPE : 0u) |
                (((ring || (WIRE && cur.kind == SRC_WIRE)) && act) ? F_CHECK : 0u);
        const uint64_t sb = (cur.sm >> e) & 1ull;
        const uint64_t si = (sb * n64 + cur.src) * L + slot;
        // wire: records {term word, slot crc, 0} at sm + 16e, payloads at sm + 16n + P·e (n = src)
        const uint8_t* sp = ring   ? p.pay + si * P
                            : wire ? p.wire + cur.sm + 16ull * cur.src + (uint64_t)P * e
                                   : p.slabs + (((uint64_t)cur.src * rows + cur.g) * p.E + e) * P;
        sp = act ? sp : dummy;
        const uint32_t* wp = (ring && act) ? &p.info[si].x
                             : (wire && act) ? reinterpret_cast<const uint32_t*>(p.wire + cur.sm + 16ull * e + 8)
                                             : reinterpret_cast<const uint32_t*>(dummy);
#ifdef RG_BULK_NT_LOAD  // ablation: non-temporal loads (r01: 1.115 vs 1.090 ms plain)
        x[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(sp + c * 16));
#else  // temporal: the second follower's read of the same leader entries hits L2 / Infinity Cache
        x[u] = *reinterpret_cast<const u32x4*>(sp + c * 16);
#endif
        want[u] = *wp;
        vmask = step ? (vmask | (1u << u)) : (vmask & ~(1u << u));
        cur.b += step ? EPI : 0u;
      }
    }
    if (cur.live && cur.b >= cur.n) cur.live = next_job<WIRE>(p, cur, tj, stride, ntiles);
  } while (rfl((uint32_t)(vmask != 0 || cur.live)));
}

static int lg_of(uint32_t P) {
  int lg = 0;
  while ((16u << lg) < P) ++lg;
  return lg;
}

int bulk_lds_bytes(uint32_t P) { return P ? (int)((CRC_T_WORDS + CRC_N_WORDS + (P / 16) * CRC_SH_STRIDE) * 4) : 16; }

template <bool W, class F>
static hipError_t with_bulk_w(uint32_t P, F f) {
  switch (lg_of(P)) {
    case 0: return f(bulk_kernel<0, W>);
    case 1: return f(bulk_kernel<1, W>);
    case 2: return f(bulk_kernel<2, W>);
    case 3: return f(bulk_kernel<3, W>);
    case 4: return f(bulk_kernel<4, W>);
    case 5: return f(bulk_kernel<5, W>);
    case 6: return f(bulk_kernel<6, W>);
    default: return hipErrorInvalidValue;
  }
}
template <class F>
static hipError_t with_bulk(uint32_t P, bool wire, F f) {
  if (!P) return hipSuccess;  // metadata-only engines have no payload stage (tick_impl)
  return wire ? with_bulk_w<true>(P, f) : with_bulk_w<false>(P, f);
}

int bulk_blocks_per_cu(uint32_t P) {
  int n = 0;
  const hipError_t r = with_bulk(P, false, [&](auto k) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 256, bulk_lds_bytes(P));
  });
  return (r == hipSuccess && n > 0) ? n : 1;
}

hipError_t launch_bulk(const BulkParams& p, hipStream_t s, int grid) {
  return with_bulk(p.P, p.wire_mode != 0, [&](auto k) {
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), bulk_lds_bytes(p.P), s, p);
    return hipGetLastError();
  });
}

// ================================================================== bootstrap (peer.go Launch + bootstrap)
__global__ void bootstrap_kernel(TickParams p, uint2* info) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= p.nrep) return;
  const uint32_t R = p.R, s = q / p.G, g = q - s * p.G;
  const uint64_t n = p.nrep;
  uint64_t* a = p.s64_out + q;
  for (uint32_t f = 0; f < S64_ROWS; ++f) a[f * n] = 0;
  uint32_t* b = p.s32_out + q;
  for (uint32_t f = 0; f < S32_ROWS; ++f) b[f * n] = 0;
  a[S_TERM * n] = 1;  // becomeFollower(1, NoLeader): one reset
  a[S_LAST * n] = R;
  a[S_COMMITTED * n] = R;
  b[S_RNG_CTR * n] = 1;
  const uint32_t im = p.IM ? p.IM : (1u << R) - 1u;  // initialMembers
  b[S_MEMBERS * n] = im;
  b[S_SNAP_MEMBERS * n] = im;
  const uint64_t key = (pl_group(p.pl, s, g) << 32) | ((uint64_t)s << 24) | 1ull;
  b[S_RAND_TO * n] = p.ET + (uint32_t)(mix64(p.seed ^ mix64(key)) % p.ET);
  for (uint32_t j = 0; j < R; ++j) {  // addNode → setRemote(id, 0, last+1)
    p.rem_out[(0 * R + j) * n + q] = 0;
    p.rem_out[(1 * R + j) * n + q] = R + 1;
    p.rem_out[(2 * R + j) * n + q] = 0;
    p.rst_out[j * n + q] = RETRY;
  }
  for (uint32_t i = 1; i <= R; ++i) {
    const uint64_t slot = i & (p.L - 1);
    p.tr[slot * n + q] = 1ull | TYPE_BIT;  // ConfigChange, term 1, no payload, bank 0
    info[(uint64_t)q * p.L + slot] = make_uint2(0u, (uint32_t)ENTRY_CONFIG << 24);
  }
  p.jcnt[q] = 0;
}

hipError_t launch_bootstrap(const TickParams& p, uint2* info, hipStream_t s) {
  hipLaunchKernelGGL(bootstrap_kernel, dim3((p.nrep + 255) / 256), dim3(256), 0, s, p, info);
  return hipGetLastError();
}

// ================================================================== proposal payload generator
// row r of a slab holds the batch of global group pl_group(s, j): r = j (one rank, rows = G) or
// r = q = s·G + j (rows = nrep: each rank's replica of a group reads its own row, so a forwarded
// proposal finds the same bytes on the leader's rank)
__global__ void fill_slabs_kernel(uint8_t* slabs, uint2* slab_info, uint32_t slab0, uint32_t nslab, uint32_t G,
                                  uint32_t rows, uint32_t E, uint32_t P, uint64_t seed, Placement pl) {
  const uint64_t wpe = P / 8;
  const uint64_t total = (uint64_t)nslab * rows * E * wpe;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < total; w += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t ent = w / wpe, wi = w - ent * wpe;
    const uint32_t i = (uint32_t)(ent % E);
    const uint64_t sg = ent / E;
    const uint32_t r = (uint32_t)(sg % rows), sl = slab0 + (uint32_t)(sg / rows);
    const uint64_t gg = pl_group(pl, r / G, r % G);
    const uint64_t key = mix64(((uint64_t)sl << 56) ^ (gg << 16) ^ (uint64_t)i ^ (seed * 0x9E3779B97F4A7C15ULL));
    const uint64_t at = (uint64_t)slab0 * rows * E * wpe + w;  // slabs [slab0, slab0 + nslab) only
    reinterpret_cast<uint64_t*>(slabs)[at] = mix64(key + (wi + 1) * 0xD1B54A32D192ED03ULL);
    if (wi == 0) slab_info[at / wpe] = make_uint2(0u, P);  // a synthetic Cmd is P bytes
  }
}

hipError_t launch_fill_slabs(uint8_t* slabs, uint2* slab_info, uint32_t slab0, uint32_t nslab, uint32_t G, uint32_t rows,
                             uint32_t E, uint32_t P, uint64_t seed, const Placement& pl, hipStream_t s) {
  if (!P) return hipSuccess;
  hipLaunchKernelGGL(fill_slabs_kernel, dim3(4096), dim3(256), 0, s, slabs, slab_info, slab0, nslab, G, rows, E, P,
                     seed, pl);
  return hipGetLastError();
}

// ================================================================== caller proposals (rg_propose)
// One wave per Cmd: lane c writes bytes [16c, 16c + 16) of the Cmd's P-byte slab slot from the caller's
// packed bytes (unaligned, read byte by byte: an H2D-staged batch, not the tick path), zero past len.
__global__ void __launch_bounds__(256) stage_cmds_kernel(uint8_t* slabs, uint2* slab_info, uint32_t P,
                                                         const uint8_t* src, const uint64_t* off, const uint64_t* dst,
                                                         const uint32_t* len, uint64_t n) {
  const uint32_t lane = __lane_id(), nch = P / 16;
  for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < n;
       i += (uint64_t)gridDim.x * (blockDim.x >> 6)) {
    const uint64_t d = dst[i], o = off[i];
    const uint32_t ln = len[i];
    for (uint32_t c = lane; c < nch; c += 64) {
      uint32_t w[4] = {0, 0, 0, 0};
      for (uint32_t b = 0; b < 16; ++b) {
        const uint32_t k = 16 * c + b;
        if (k < ln) w[b >> 2] |= (uint32_t)src[o + k] << (8 * (b & 3));
      }
      *reinterpret_cast<uint4*>(slabs + d * P + 16ull * c) = make_uint4(w[0], w[1], w[2], w[3]);
    }
    if (lane == 0) slab_info[d] = make_uint2(0u, ln);
  }
}

hipError_t launch_stage_cmds(uint8_t* slabs, uint2* slab_info, uint32_t P, const uint8_t* src, const uint64_t* off,
                             const uint64_t* dst, const uint32_t* len, uint64_t n, hipStream_t s) {
  if (!n || !P) return hipSuccess;
  const uint64_t blocks = std::min<uint64_t>((n + 3) / 4, 65536);
  hipLaunchKernelGGL(stage_cmds_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, slabs, slab_info, P, src, off, dst,
                     len, n);
  return hipGetLastError();
}

// ================================================================== kernel-argument placement probe (tests)
__global__ void kernarg_probe_kernel(uint64_t* out, uint64_t tag) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out[0] = (uint64_t)(uintptr_t)__builtin_amdgcn_kernarg_segment_ptr();
    out[1] = tag;
  }
}

hipError_t launch_kernarg_probe(uint64_t* out, uint64_t tag, hipStream_t s) {
  hipLaunchKernelGGL(kernarg_probe_kernel, dim3(1), dim3(64), 0, s, out, tag);
  return hipGetLastError();
}

// ================================================================== copy probe (measurement)
// The fastest of the shapes scripts/copy_probe.hip measured on MI355X (r01: 5.94 TB/s read + write):
// one block per 32-KB tile, eight 16-B non-temporal loads in flight per lane.
__global__ void __launch_bounds__(256) probe_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                         uint64_t n) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint64_t b = (uint64_t)blockIdx.x * 2048;
  u32x4 v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const uint64_t i = b + u * 256 + threadIdx.x;
    v[u] = i < n ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + i)) : u32x4{0, 0, 0, 0};
  }
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const uint64_t i = b + u * 256 + threadIdx.x;
    if (i < n) __builtin_nontemporal_store(v[u], reinterpret_cast<u32x4*>(dst + i));
  }
}

hipError_t launch_probe_copy(const void* src, void* dst, uint64_t bytes, hipStream_t s) {
  const uint64_t n = bytes / 16;
  hipLaunchKernelGGL(probe_copy_kernel, dim3((uint32_t)((n + 2047) / 2048)), dim3(256), 0, s, (const uint4*)src,
                     (uint4*)dst, n);
  return hipGetLastError();
}

// ================================================================== reductions
__device__ __forceinline__ uint64_t wave_sum64(uint64_t a) {
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)a, off, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(a >> 32), off, 64);
    a += ((uint64_t)hi << 32) | lo;
  }
  return a;
}

// Σ_g max_s committed, on the state a next tick would read (s64_in). With ranks > 1 the replicas
// of a column belong to different groups: sum the slot-0 replicas hosted here (each group's slot 0
// lives on exactly one rank, so the sum over ranks counts every group once).
__global__ void sum_committed_kernel(TickParams p, unsigned long long* out) {
  uint64_t acc = 0;
  const uint32_t ns = p.pl.N > 1 ? 1u : p.R;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < p.G; g += gridDim.x * blockDim.x) {
    uint64_t m = 0;
    for (uint32_t s = 0; s < ns; ++s) m = umax64(m, p.s64_in[(uint64_t)S_COMMITTED * p.nrep + (uint64_t)s * p.G + g]);
    acc += m;
  }
  acc = wave_sum64(acc);
  if (lane_id() == 0 && acc) atomicAdd(out, (unsigned long long)acc);
}

hipError_t launch_sum_committed(const TickParams& p, unsigned long long* out, hipStream_t s) {
  hipLaunchKernelGGL(sum_committed_kernel, dim3(256), dim3(256), 0, s, p, out);
  return hipGetLastError();
}

// Last tick's traffic: leaders, msgs, replicate entries, appended, leader-appended.
// p is the parameter block a next tick would use: s64_in = current state, s64_out = previous
// state, cnt_in/hdr_in = the last tick's outbox.
__global__ void traffic_kernel(TickParams p, unsigned long long* out6) {
  uint64_t v[5] = {0, 0, 0, 0, 0};
  const uint64_t n = p.nrep;
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < p.nrep; q += gridDim.x * blockDim.x) {
    const uint32_t s = q / p.G, g = q - s * p.G;
    const bool ld = p.s32_in[S_ROLE * n + q] == LEADER;
    v[0] += ld;
    for (uint32_t d = 0; d < p.R; ++d) {
      const uint32_t c = p.cnt_in[((uint64_t)s * p.R + d) * p.G + g];
      v[1] += c;
      for (uint32_t k = 0; k < c; ++k) {
        const uint64_t w0 = p.hdr_in[(((uint64_t)s * p.R + d) * p.K + k) * p.G + g];
        if ((w0 & 0xFF) == M_REPLICATE) v[2] += w0 >> 32;
      }
    }
    const uint64_t lc = p.s64_in[S_LAST * n + q], lp = p.s64_out[S_LAST * n + q];
    const uint64_t app = lc > lp ? lc - lp : 0;
    v[3] += app;
    if (ld) v[4] += app;
  }
  for (int i = 0; i < 5; ++i) {
    const uint64_t a = wave_sum64(v[i]);
    if (lane_id() == 0 && a) atomicAdd(out6 + i, (unsigned long long)a);
  }
}

hipError_t launch_traffic(const TickParams& p, unsigned long long* out6, hipStream_t s) {
  hipLaunchKernelGGL(traffic_kernel, dim3(512), dim3(256), 0, s, p, out6);
  return hipGetLastError();
}

}  // namespace rg
