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
#include <type_traits>
#include <cstdlib>

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
// copy (DESIGN.md §3 "The control-kernel fault"). Before anything is dereferenced, every lane checks
// the block's checksum (uniform scalar loads): a stale or torn block becomes a sticky engine error
// (*perr, a separate kernel argument, reported by the next synchronising call) instead of wild
// addresses. Ctl reads the fields in place.
template <int R>
__global__ void __launch_bounds__(RG_CTL_BLOCK, RG_CTL_MINWAVES) control_kernel(const TickParams* __restrict__ pp,
                                                                               uint32_t* perr) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  // The checksum: lane i loads word i (one coalesced 424-B wave load, through a laundered pointer so
  // it stays separate from the step's scalar field reads) and the wave sums the terms with a
  // butterfly. r03a's volatile chain cost 53 dependent cache-bypassing loads per wave; a chain of
  // seven s_load_dwordx16 (r03b) still waited seven scalar round trips at the head of every wave.
  const TickParams* pc = pp;
  asm volatile("" : "+s"(pc));
  const uint32_t lane = threadIdx.x & 63u;
  typedef __attribute__((address_space(1))) const uint64_t gu64;
  gu64* wv = (gu64*)pc;  // a C cast: the address-space conversion (global_load, not flat_load)
  uint64_t h = lane < TP_WORDS ? tp_term(wv[lane], lane) : 0ull;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)h, off, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(h >> 32), off, 64);
    h += ((uint64_t)hi << 32) | lo;
  }
  if (h != wv[TP_WORDS]) {
    if (q == 0) {
      printf("raftgpu: control_kernel parameter block checksum mismatch (tick %llu): launch skipped\n",
             (unsigned long long)pp->tick);
      atomicOr(perr, 1u);
    }
    return;
  }
  CTickParams& cp = *(CTickParams*)pp;
  if (q >= cp.nrep) return;
#ifdef RG_CTL_PROFILE
  const uint32_t t0 = (uint32_t)__builtin_amdgcn_s_memtime();
  Ctl<R> c(cp, q);
  c.stamps[0] = t0;
#else
  Ctl<R> c(cp, q);
#endif
  c.run();
}

// ---- the resident multi-tick control kernel (metadata-only, one-rank engines). A
// workgroup holds every replica of 64 groups — wave w is slot w of groups [64·b, 64·b + 64) — so a
// tick's messages never leave it, and k ticks run in one launch with a workgroup barrier between
// them instead of a kernel boundary: the state, outboxes and ring words a tick reads were written
// by this workgroup one tick earlier and are still in its CU's caches. Block i of pp is tick t0 + i
// (the host seals each); all k checksums are verified before anything is dereferenced.
__device__ __forceinline__ bool tp_check(const TickParams* pp, uint32_t i) {
  const TickParams* pc = pp + i;
  asm volatile("" : "+s"(pc));
  typedef __attribute__((address_space(1))) const uint64_t gu64;
  gu64* wv = (gu64*)pc;
  const uint32_t lane = threadIdx.x & 63u;
  uint64_t h = lane < TP_WORDS ? tp_term(wv[lane], lane) : 0ull;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)h, off, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(h >> 32), off, 64);
    h += ((uint64_t)hi << 32) | lo;
  }
  return h == wv[TP_WORDS];
}

template <int R>
__global__ void __launch_bounds__(64 * R, 1) control_resident_kernel(const TickParams* __restrict__ pp, uint32_t k,
                                                                     uint32_t* perr) {
  for (uint32_t i = 0; i < k; ++i)
    if (!tp_check(pp, i)) {  // the same verdict in every wave: the whole workgroup leaves together
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        printf("raftgpu: control_resident_kernel parameter block %u checksum mismatch: launch skipped\n", i);
        atomicOr(perr, 1u);
      }
      return;
    }
  CTickParams* cp = (CTickParams*)pp;
  const uint32_t G = cp[0].G, w = threadIdx.x >> 6, g = blockIdx.x * 64 + (threadIdx.x & 63u);
  const uint32_t q = w * G + g;
  for (uint32_t i = 0; i < k; ++i) {
    if (g < G) {
      Ctl<R> c(cp[i], q);
      c.run();
    }
    __syncthreads();  // tick i's outboxes and state, written by this workgroup, before tick i + 1 reads them
  }
}

hipError_t launch_control_resident(const TickParams* p, uint32_t k, uint32_t* perr, uint32_t R, uint32_t G,
                                   hipStream_t s) {
#ifdef RG_DEV_NO_CONTROL
  (void)p; (void)k; (void)perr; (void)R; (void)G; (void)s;
  return hipErrorInvalidValue;
#endif
  dim3 grid((G + 63) / 64), block(64 * R);
  switch (R) {
    case 1: hipLaunchKernelGGL(control_resident_kernel<1>, grid, block, 0, s, p, k, perr); break;
    case 2: hipLaunchKernelGGL(control_resident_kernel<2>, grid, block, 0, s, p, k, perr); break;
    case 3: hipLaunchKernelGGL(control_resident_kernel<3>, grid, block, 0, s, p, k, perr); break;
    case 4: hipLaunchKernelGGL(control_resident_kernel<4>, grid, block, 0, s, p, k, perr); break;
    // R > 4: a control wave needs a SIMD of its own (occupancy 1), and a CU has four
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_control(const TickParams* p, uint32_t* perr, uint32_t R, uint32_t nrep, hipStream_t s) {
  dim3 grid((nrep + RG_CTL_BLOCK - 1) / RG_CTL_BLOCK), block(RG_CTL_BLOCK);
#ifdef RG_DEV_NO_CONTROL  // development builds of the other kernels only (ISA / resource checks)
  (void)grid; (void)block; (void)p; (void)perr; (void)R; (void)s;
  return hipErrorInvalidValue;
#endif
  switch (R) {
    case 1: hipLaunchKernelGGL(control_kernel<1>, grid, block, 0, s, p, perr); break;
    case 2: hipLaunchKernelGGL(control_kernel<2>, grid, block, 0, s, p, perr); break;
    case 3: hipLaunchKernelGGL(control_kernel<3>, grid, block, 0, s, p, perr); break;
    case 4: hipLaunchKernelGGL(control_kernel<4>, grid, block, 0, s, p, perr); break;
    case 5: hipLaunchKernelGGL(control_kernel<5>, grid, block, 0, s, p, perr); break;
    case 6: hipLaunchKernelGGL(control_kernel<6>, grid, block, 0, s, p, perr); break;
    case 7: hipLaunchKernelGGL(control_kernel<7>, grid, block, 0, s, p, perr); break;
    case 8: hipLaunchKernelGGL(control_kernel<8>, grid, block, 0, s, p, perr); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ================================================================== bulk kernel
struct Crc {
  const uint32_t* T;   // LDS [16][256] byte tables
  const uint32_t* N;   // LDS [16][2][16] nibble tables
  const uint32_t* SH;  // LDS this lane's [8][16] shift table
  const uint32_t* ZP;  // LDS [8][16] Z^P (a Cmd longer than P: chaining its P-byte segments)
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
  // Z^(16·(NCH−1−c))(v): move this lane's chunk contribution to the end of its P-byte segment
  __device__ __forceinline__ uint32_t shift(uint32_t v) const {
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r ^= SH[j * 16 + ((v >> (4 * j)) & 0xF)];
    return r;
  }
  __device__ __forceinline__ uint32_t zp(uint32_t v) const {
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r ^= ZP[j * 16 + ((v >> (4 * j)) & 0xF)];
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

__device__ __forceinline__ uint32_t wave_excl_scan32(uint32_t v) {
  const uint32_t lane = lane_id();
  uint32_t x = v;
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
    if (lane >= o) x += y;
  }
  return x - v;
}

#ifndef RG_BULK_U
#define RG_BULK_U 4
#endif
constexpr int BULK_U = RG_BULK_U;  // 16-B chunks in flight per lane

// One copy job, its fields uniform across the wave (SGPRs): n entries from `first`, payloads
// from the sender's stream, a proposal slab / Cmd arena or the receive buffer into this replica's
// stream, CRC per entry (raftgpu_internal.h: job rows).
struct Job {
  uint64_t first, spos, sm, dm;
  uint32_t meta, src, dpos;
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
  jb.spos = p.job64[J_SPOS * JN + jq];
  jb.sm = p.job64[J_SMASK * JN + jq];
  jb.dm = p.job64[J_DMASK * JN + jq];
  jb.meta = p.job32[J_META * JN + jq];
  jb.src = p.job32[J_SRC * JN + jq];
  jb.dpos = p.job32[J_DPOS * JN + jq];
  return jb;
}

// ---- software-pipelined payload stream.
// A wave walks a flat sequence of steps over the jobs of its tiles; one step = epi entries of one
// uniform job, 16 B per lane. BULK_U steps are in flight at once in a register ring: slot u is
// consumed (store, CRC, info, verify) and immediately re-issued with the step BULK_U ahead. All
// cursor state is wave-uniform (SGPRs). A non-uniform job drains the ring and runs on its own
// (vjob: per-entry source positions, Cmds of any length).
struct Cursor {
  uint32_t t, q, qb, g, njl, j, n, kind, src, b, e0, ncu, dpos;
  uint64_t m, first, spos, sm, dm;
  bool live, uni;
};

struct TileJobs {  // per lane: job count and first job of replica qb + lane
  uint32_t nj;
  Job j0;
  uint32_t pd0, pd1, ps0, ps1;  // MJ: page ids of that job's first step
};

// the page ids a job's first step needs: destination pages vpn(dpos), +1; a ring job's source
// pages vpn(spos + e0 * ncu), +1 (the page tables are fixed during the launch)
__device__ __forceinline__ void first_step_pages(const BulkParams& p, const uint32_t* __restrict__ pt, uint32_t q,
                                                 const Job& jb, uint32_t& pd0, uint32_t& pd1, uint32_t& ps0,
                                                 uint32_t& ps1) {
  const uint32_t PTSM = p.PTS - 1, ncu = (jb.meta >> 21) & 0x7F, e0 = (jb.meta >> 8) & 0xFF;
  const uint32_t kind = (jb.meta >> 16) & 0xF, dv = vpn_of(jb.dpos);
  const uint64_t dr = (uint64_t)q * p.PTS;
  pd0 = pt[dr + (dv & PTSM)];
  pd1 = pt[dr + ((dv + 1) & PTSM)];
  ps0 = ps1 = 0;
  if (kind == SRC_RING && jb.src < p.nrep) {
    const uint32_t sv = vpn_of((uint32_t)jb.spos + e0 * ncu);
    const uint64_t sr = (uint64_t)jb.src * p.PTS;
    ps0 = pt[sr + (sv & PTSM)];
    ps1 = pt[sr + ((sv + 1) & PTSM)];
  }
}

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

template <bool MJ = false>
__device__ __forceinline__ void load_tile(const BulkParams& p, Cursor& cur, TileJobs& tj,
                                          const uint32_t* __restrict__ pt = nullptr) {
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
  tj.pd0 = tj.pd1 = tj.ps0 = tj.ps1 = 0;
#ifdef RG_BULK_MJ_PF
  if constexpr (MJ) {  // one more round trip per tile instead of one per job (C5: one-entry jobs)
    if (tj.nj) first_step_pages(p, pt, q, tj.j0, tj.pd0, tj.pd1, tj.ps0, tj.ps1);
  }
#else
  (void)pt;
#endif
  cur.m = __ballot(tj.nj != 0);
  cur.j = 0;
  cur.njl = 0;
}

template <int LG, bool WIRE>
__device__ __forceinline__ void set_job(const BulkParams& p, Cursor& cur, const Job& jb) {
  constexpr uint32_t NCH = 1u << LG;
  cur.first = jb.first; cur.spos = jb.spos; cur.sm = jb.sm; cur.dm = jb.dm; cur.dpos = jb.dpos;
  cur.n = jb.meta & 0xFF; cur.b = (jb.meta >> 8) & 0xFF; cur.e0 = cur.b; cur.kind = (jb.meta >> 16) & 0xF;
  cur.uni = (jb.meta >> 20) & 1; cur.ncu = (jb.meta >> 21) & 0x7F;
  cur.src = jb.src;
  const bool slab = cur.kind == SRC_SLAB || cur.kind == SRC_CMD;
  cur.g = WIRE ? (cur.src >> 16) * p.G + cur.q % p.G : cur.q % p.G;  // SRC_SLAB / SRC_CMD: the batch's slab row
  if (slab) cur.src &= 0xFFFFu;
  const bool wk = cur.kind == SRC_WIRE || cur.kind == SRC_WIRE_PROP;
  // a malformed job (never produced by control_kernel) is skipped and marks its replica ERR_WIRE
  const bool bad =
      cur.n > 64 || cur.e0 > cur.n || cur.kind > SRC_CMD || (cur.uni && cur.ncu > NCH) ||
      (cur.kind == SRC_SLAB && (!cur.uni || cur.ncu != NCH)) || (cur.kind == SRC_RING && cur.src >= p.nrep) ||
      (slab && (cur.src >= p.nslab || cur.g >= (WIRE ? p.nrep : p.G))) ||
      (wk && (!p.wire_mode || cur.n > cur.src || cur.spos + 16ull * cur.src > p.wire_bytes ||
              (cur.uni && (cur.e0 != 0 || cur.spos + 16ull * cur.src * (1 + cur.ncu) > p.wire_bytes)))) ||
      (cur.kind == SRC_CMD && cur.uni && (cur.spos + (uint64_t)(cur.n - cur.e0) * cur.ncu) * 16 > p.cmd_cap);
  if (bad) {
#ifdef RG_BOUNDS
    if (lane_id() == 0)
      printf("RG_BOUNDS bulk q=%u job=%u n=%u e0=%u kind=%u src=%u spos=%llu wire_bytes=%llu\n", cur.q, cur.j, cur.n,
             cur.e0, cur.kind, cur.src, (unsigned long long)cur.spos, (unsigned long long)p.wire_bytes);
#endif
    if (lane_id() == 0) atomicOr(p.crc_err + cur.q, ERR_WIRE);
    cur.n = 0;
    cur.b = cur.e0 = 0;
    cur.uni = true;
  }
}

// Move the cursor one position: the replica's next job, the tile's next replica, or the next
// tile (whose descriptors arrive in one round trip; that pass issues nothing). A job with no
// entries left to write simply yields an empty pass. Returns false once the wave is done.
template <int LG, bool WIRE, bool MJ = false>
__device__ __forceinline__ bool next_job(const BulkParams& p, Cursor& cur, TileJobs& tj, uint32_t stride,
                                         uint32_t ntiles, const uint32_t* __restrict__ pt = nullptr) {
  if (cur.j + 1 < cur.njl) {
    ++cur.j;
    set_job<LG, WIRE>(p, cur, load_job(p, cur.q, cur.j));
  } else if (cur.m) {
    const uint32_t l = rfl((uint32_t)__ffsll((long long)cur.m) - 1);
    cur.m &= cur.m - 1;
    cur.q = cur.qb + l;
    cur.njl = __builtin_amdgcn_readlane(tj.nj, l);
    cur.j = 0;
    Job jb;
    jb.first = rl64(tj.j0.first, l); jb.spos = rl64(tj.j0.spos, l); jb.sm = rl64(tj.j0.sm, l);
    jb.dm = rl64(tj.j0.dm, l);
    jb.meta = __builtin_amdgcn_readlane(tj.j0.meta, l); jb.src = __builtin_amdgcn_readlane(tj.j0.src, l);
    jb.dpos = __builtin_amdgcn_readlane(tj.j0.dpos, l);
    set_job<LG, WIRE>(p, cur, jb);
  } else {
    cur.t += stride;
    if (cur.t >= ntiles) return false;
    load_tile<MJ>(p, cur, tj, pt);
    cur.b = 0;  // two statements: the chained form kept Cursor in scratch
    cur.n = 0;
    cur.uni = true;
  }
  return true;
}

// The tile's next replica, from the first-job descriptors the tile load left in registers: no
// memory round trip, so the cursor can take it in the middle of a pass (small jobs share a pass).
template <int LG, bool WIRE>
__device__ __forceinline__ void next_replica(const BulkParams& p, Cursor& cur, const TileJobs& tj) {
  const uint32_t l = rfl((uint32_t)__ffsll((long long)cur.m) - 1);
  cur.m &= cur.m - 1;
  cur.q = cur.qb + l;
  cur.njl = __builtin_amdgcn_readlane(tj.nj, l);
  cur.j = 0;
  Job jb;
  jb.first = rl64(tj.j0.first, l); jb.spos = rl64(tj.j0.spos, l); jb.sm = rl64(tj.j0.sm, l);
  jb.dm = rl64(tj.j0.dm, l);
  jb.meta = __builtin_amdgcn_readlane(tj.j0.meta, l); jb.src = __builtin_amdgcn_readlane(tj.j0.src, l);
  jb.dpos = __builtin_amdgcn_readlane(tj.j0.dpos, l);
  set_job<LG, WIRE>(p, cur, jb);
}

// the entry info word {slot crc, stream position} (and the sender-CRC check) at ring slot `slot`,
// info bank `bank`
__device__ __forceinline__ void put_info_at(const BulkParams& p, uint32_t q, uint64_t slot, uint64_t bank, uint32_t crc,
                                            uint32_t pos, bool check, uint32_t want) {
  p.info[(bank * p.nrep + q) * p.L + slot] = make_uint2(crc, pos);
  if (check && want != crc) atomicOr(p.crc_err + q, ERR_CRC);
}

// the entry info word {slot crc, stream position} (and the sender-CRC check) of job entry e
__device__ __forceinline__ void put_info(const BulkParams& p, uint32_t q, uint64_t first, uint64_t dm, uint32_t e,
                                         uint32_t crc, uint32_t pos, bool check, uint32_t want) {
  const uint64_t slot = (first + e) & (p.L - 1), bank = (dm >> e) & 1ull;
  p.info[(bank * p.nrep + q) * p.L + slot] = make_uint2(crc, pos);
  if (check && want != crc) atomicOr(p.crc_err + q, ERR_CRC);
}

// A non-uniform job (Cmds of different lengths, a Replicate the sender built from its ring, caller
// Cmds, Cmds longer than P): lane e reads entry e's source position and length, a wave scan lays
// the Cmds out back to back from J_DPOS, then up to 64/NCH entries of at most P bytes move per
// pass (NCH lanes each, as in the uniform path), and a longer Cmd moves alone, 64 chunks per pass,
// its P-byte segments' CRCs chained with Z^P. Page-table lookups are per lane (not pipelined).
template <int LG, bool WIRE>
__device__ void vjob(const BulkParams& p, const uint32_t* __restrict__ pt, const Cursor& cur, const Crc& crc) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  constexpr uint32_t NCH = 1u << LG, EPI = 64u >> LG;
  const uint32_t lane = lane_id(), c = lane & (NCH - 1), ei = lane >> LG;
  const uint32_t n = cur.n, e0 = cur.e0, q = cur.q, kind = cur.kind;
  const uint64_t n64 = p.nrep, L = p.L, PTS = p.PTS;
  const bool ring = kind == SRC_RING, wire = WIRE && (kind == SRC_WIRE || kind == SRC_WIRE_PROP);
  const bool check = ring || (WIRE && kind == SRC_WIRE);
  const uint64_t rows = WIRE ? p.nrep : p.G;
  const uint8_t* arena = p.cmds + (uint64_t)cur.src * p.cmd_cap;
  const uint64_t wpay = cur.spos + 16ull * n;  // wire: payload base
  // lane e: entry e's chunks, source position (sender stream / arena / wire chunk) and sender CRC
  const uint32_t e = lane;
  const bool in = e >= e0 && e < n;
  uint32_t nc = 0, sp = 0, want = 0;
  if (in) {
    const uint64_t slot = (cur.first + e) & (L - 1);
    nc = word_nc(p.tr[slot * n64 + q]);
    if (ring) {
      const uint2 inf = p.info[(((cur.sm >> e) & 1ull) * n64 + cur.src) * L + slot];
      want = inf.x;
      sp = inf.y;
    } else if (wire) {
      const uint32_t* r = reinterpret_cast<const uint32_t*>(p.wire + cur.spos + 16ull * e);
      want = r[2];
      sp = r[3];
      if (wpay + ((uint64_t)sp + nc) * 16 > p.wire_bytes) nc = sp = 0;  // validated by unpack; never here
    } else if (kind == SRC_CMD) {
      sp = p.slab_info[((uint64_t)cur.src * rows + cur.g) * p.E + e].x;
      if (((uint64_t)sp + nc) * 16 > p.cmd_cap) nc = sp = 0;
    } else {
      nc = 0;
    }
  }
  const uint32_t dpe = cur.dpos + wave_excl_scan32(nc);
  const uint64_t bigm = __ballot(in && nc > NCH);
  auto src_at = [&](uint32_t pos) -> const uint8_t* {
    return ring ? p.pool + stream_byte(pt, p.PTS, cur.src, pos)
           : wire ? p.wire + wpay + 16ull * pos
                  : arena + 16ull * pos;
  };
  uint32_t ee = e0;
  while (ee < n) {
    const uint32_t nce = __builtin_amdgcn_readlane(nc, ee);
    if (nce > NCH) {  // one Cmd longer than P
      const uint32_t spe = __builtin_amdgcn_readlane(sp, ee), dpee = __builtin_amdgcn_readlane(dpe, ee);
      uint32_t acc = 0;
      for (uint32_t w0 = 0; w0 < nce; w0 += 64) {
        const uint32_t k = w0 + lane;
        u32x4 x = u32x4{0, 0, 0, 0};
        if (k < nce) {
          x = *reinterpret_cast<const u32x4*>(src_at(spe + k));
          *reinterpret_cast<u32x4*>(p.pool + stream_byte(pt, p.PTS, q, dpee + k)) = x;
        }
        uint32_t v = crc.raw16(make_uint4(x.x, x.y, x.z, x.w));
        if constexpr (LG > 0) v = xor_lanes<LG>(crc.shift(v));
        for (uint32_t gi = 0; gi < EPI && w0 + gi * NCH < nce; ++gi)
          acc = crc.zp(acc) ^ (uint32_t)__builtin_amdgcn_readlane(v, gi * NCH);
      }
      const uint32_t S = (nce + NCH - 1) / NCH;
      const uint32_t cr = p.crc_tab[CRC_CS_OFF + (S <= CRC_CS_MAX ? S : CRC_CS_MAX)] ^ acc;
      const uint32_t we = __builtin_amdgcn_readlane(want, ee);
      if (lane == 0) put_info(p, q, cur.first, cur.dm, ee, cr, dpee, check, we);
      ++ee;
    } else {  // up to EPI consecutive Cmds of at most P bytes, NCH lanes each
      uint32_t kk = n - ee < EPI ? n - ee : EPI;
      const uint64_t bb = bigm >> ee;
      if (bb) kk = min(kk, (uint32_t)__ffsll((long long)bb) - 1);
      const uint32_t me = ee + ei;
      const bool grp = ei < kk;
      const uint32_t mnc = (uint32_t)__shfl((int)nc, (int)me, 64), msp = (uint32_t)__shfl((int)sp, (int)me, 64);
      const uint32_t mdp = (uint32_t)__shfl((int)dpe, (int)me, 64), mw = (uint32_t)__shfl((int)want, (int)me, 64);
      const bool act = grp && c < mnc;
      u32x4 x = u32x4{0, 0, 0, 0};
      if (act) {
        x = *reinterpret_cast<const u32x4*>(src_at(msp + c));
        *reinterpret_cast<u32x4*>(p.pool + stream_byte(pt, p.PTS, q, mdp + c)) = x;
      }
      uint32_t v = crc.raw16(make_uint4(x.x, x.y, x.z, x.w));
      if constexpr (LG > 0) v = xor_lanes<LG>(crc.shift(v));
      if (grp && c == 0) put_info(p, q, cur.first, cur.dm, me, mnc ? p.crc_const ^ v : 0u, mdp, check && mnc, mw);
      ee += kk;
    }
  }
  (void)PTS;
}

// P = 16 << LG bytes per lane group: 2^LG lanes per entry (16 B each), 64 >> LG entries per step.
// WIRE: the engine exchanges messages with other ranks (SRC_WIRE jobs, slab rows per replica);
// one-rank engines run the variant without those paths.
// MJ: small jobs share a pass — a ring slot takes the tile's next replica's job as soon as the current
// one is issued (C5's one-entry jobs: bulk 3.99 -> 1.67 ms). It costs the 64-entry jobs of the
// 64K x 3 workload 8% (1.26 -> 1.36 ms, r03f A/B), so the host picks it per engine (launch_bulk).
#ifdef RG_BULK_WPE  // A/B: hold the compiler to RG_BULK_WPE waves per SIMD
#define RG_BULK_ATTR __attribute__((amdgpu_waves_per_eu(RG_BULK_WPE, RG_BULK_WPE)))
#else
#define RG_BULK_ATTR
#endif
template <int LG, bool WIRE, bool MJ>
__global__ void __launch_bounds__(256) RG_BULK_ATTR bulk_kernel(BulkParams p, const uint32_t* __restrict__ pt) {
  constexpr uint32_t NCH = 1u << LG, EPI = 64u >> LG, P = 16u << LG;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t shw = CRC_T_WORDS + CRC_N_WORDS + NCH * CRC_SH_STRIDE;
  for (uint32_t i = threadIdx.x; i < shw; i += blockDim.x) lds[i] = p.crc_tab[i];
  for (uint32_t i = threadIdx.x; i < CRC_ZP_WORDS; i += blockDim.x) lds[shw + i] = p.crc_tab[CRC_ZP_OFF + i];
  // pages freed by this tick's pool kernel become allocatable from the next tick on
  if (blockIdx.x == 0 && threadIdx.x == 0) p.poolctl->limit = p.poolctl->tail;
  __syncthreads();
  const uint32_t waves = blockDim.x >> 6, lane = lane_id();
  const uint32_t stride = gridDim.x * waves;
  const uint32_t ntiles = bulk_ntiles(p);
  const uint64_t n64 = p.nrep, L = p.L, rows = WIRE ? p.nrep : p.G;
  const uint32_t PTSM = p.PTS - 1;
  const uint32_t c = lane & (NCH - 1), ei = lane >> LG;
  const Crc crc{lds, lds + CRC_T_WORDS, lds + CRC_T_WORDS + CRC_N_WORDS + c * CRC_SH_STRIDE, lds + shw};
  Cursor cur{};
  TileJobs tj{};
  cur.t = rfl(blockIdx.x * waves + (threadIdx.x >> 6));
  if (cur.t >= ntiles) return;
  load_tile<MJ>(p, cur, tj, pt);
  cur.b = 0;  // two statements: the chained form kept Cursor in scratch
  cur.n = 0;
  cur.uni = true;
  cur.live = next_job<LG, WIRE, MJ>(p, cur, tj, stride, ntiles, pt);
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  // Two ring walks: MJ keeps each slot's job in scalars and lets a slot take the tile's next
  // replica mid-pass (small jobs); without MJ the slots of a pass share one job (per-pass scalars,
  // fewer SGPRs: the 64-entry jobs of full batches run faster so).
  if constexpr (MJ) {
  // ring slot u: payload chunk, destination pool chunk, sender's slot CRC (per lane). The job a slot's
  // step belongs to is wave-uniform and kept per slot (scalars): replica sq, first index sfirst, bank
  // mask sdm, first entry of the step sb, job start se0 / destination chunk sdp / chunks per entry
  // sncu, entries in the step skv (0 = empty), whether followers check the sender CRC schk. A slot
  // may take the tile's next replica's job in the middle of a pass (from registers, no round trip),
  // so a pass of small jobs (C5: one entry per job) fills all BULK_U slots instead of one.
  u32x4 x[BULK_U];
  uint32_t ds[BULK_U], want[BULK_U];
  // sm[u] packs the small fields: step's first entry b (7 bits) | job start e0 << 7 | chunks per
  // entry ncu << 14 | entries in the step << 21 | check << 28 (fewer scalars: fewer SGPR spills)
  // ss[u] = the ring slot of the step's first entry, sbk[u] = the step's destination bank bits (one
  // per entry, EPI of them)
  typedef std::conditional_t<(EPI <= 32), uint32_t, uint64_t> Banks;
  uint32_t sq[BULK_U], sdp[BULK_U], sm[BULK_U], ss[BULK_U];
  Banks sbk[BULK_U];
#pragma unroll
  for (int u = 0; u < BULK_U; ++u) {
    x[u] = u32x4{0, 0, 0, 0};
    ds[u] = want[u] = 0;
    sq[u] = sdp[u] = sm[u] = ss[u] = 0;
    sbk[u] = 0;
  }
  // Every slot issues exactly two loads per pass (payload chunk + sender CRC word), redirected to a
  // dummy address when the slot has no work, so the number of memory operations between a load
  // and its use is the same on every path and the compiler's vmcnt waits keep the ring in flight.
  const uint8_t* dummy = reinterpret_cast<const uint8_t*>(p.crc_tab + CRC_ZERO_OFF);  // 16 zero bytes
  uint32_t vmask = 0;
  do {
#pragma unroll
    for (int u = 0; u < BULK_U; ++u) {
      {  // consume slot u: store, CRC, info, verify (no entries: no stores). A stream's Cmd is followed
        // by zeros up to its chunk boundary (every writer copies whole chunks), and lanes past a Cmd's
        // chunks contribute nothing, so the CRC is the slot CRC.
        const uint32_t sb = sm[u] & 0x7Fu, se0 = (sm[u] >> 7) & 0x7Fu, sncu = (sm[u] >> 14) & 0x7Fu;
        const uint32_t skv = (sm[u] >> 21) & 0x7Fu;
        const bool schk = (sm[u] >> 28) & 1u;
        const bool valid = ei < skv;
        const bool act = valid && c < sncu;
        if (act) {
#ifdef RG_BULK_PLAIN_STORE
          *reinterpret_cast<u32x4*>(p.pool + (uint64_t)ds[u] * 16) = x[u];
#else
          __builtin_nontemporal_store(x[u], reinterpret_cast<u32x4*>(p.pool + (uint64_t)ds[u] * 16));
#endif
        }
        uint32_t v = 0;
#ifndef RG_BULK_NOCRC
        v = crc.raw16(make_uint4(x[u].x, x[u].y, x[u].z, x[u].w));
#endif
        if constexpr (LG > 0) v = xor_lanes<LG>(crc.shift(v));  // raw(slot) = XOR_c Z^(after c)(raw c)
        if (valid && c == 0) {
          const uint32_t e = sb + ei;
          put_info_at(p, sq[u], (ss[u] + ei) & (L - 1), (sbk[u] >> ei) & 1u, act ? (p.crc_const ^ v) : 0u,
                      sdp[u] + (e - se0) * sncu, schk && act, want[u]);
        }
      }
      {  // issue the job's next step (or an empty step) into slot u
        // a uniform job fully issued: take the tile's next replica now if that costs no round trip
        if (cur.live && cur.uni && cur.b >= cur.n && cur.j + 1 >= cur.njl && cur.m)
          next_replica<LG, WIRE>(p, cur, tj);
        const bool step = cur.live && cur.uni && cur.b < cur.n;
        const uint32_t e = cur.b + ei;
        const bool valid = step && e < cur.n;
        const bool act = valid && c < cur.ncu;
        const bool ring = cur.kind == SRC_RING, wire = WIRE && (cur.kind == SRC_WIRE || cur.kind == SRC_WIRE_PROP);
        // destination chunks of this step: at most 64, so at most two stream pages (page ids by
        // scalar loads: uniform addresses)
        const uint32_t d0 = cur.dpos + (cur.b - cur.e0) * cur.ncu, dv = vpn_of(d0);
        const uint32_t dl = d0 + ei * cur.ncu + c;
        uint32_t pd0 = 0, pd1 = 0, ps0 = 0, ps1 = 0;
        const uint32_t s0 = (uint32_t)cur.spos + cur.b * cur.ncu, sv = vpn_of(s0);
#ifdef RG_BULK_MJ_PF
        // a replica's first job (cur.j 0) came from the tile load, which also fetched its first
        // step's page ids (lane q - qb of tj): no scalar round trip when this step is that step's pages
        if (step && cur.ncu && cur.j == 0 && dv == vpn_of(cur.dpos) &&
            (!ring || sv == vpn_of((uint32_t)cur.spos + cur.e0 * cur.ncu))) {
          const uint32_t l = cur.q - cur.qb;
          pd0 = __builtin_amdgcn_readlane(tj.pd0, l);
          pd1 = __builtin_amdgcn_readlane(tj.pd1, l);
          ps0 = __builtin_amdgcn_readlane(tj.ps0, l);
          ps1 = __builtin_amdgcn_readlane(tj.ps1, l);
        } else
#endif
        if (step && cur.ncu) {
          const uint64_t dr = (uint64_t)cur.q * p.PTS;
          pd0 = pt[dr + (dv & PTSM)];
          pd1 = pt[dr + ((dv + 1) & PTSM)];
          if (ring) {
            const uint64_t sr = (uint64_t)cur.src * p.PTS;
            ps0 = pt[sr + (sv & PTSM)];
            ps1 = pt[sr + ((sv + 1) & PTSM)];
          }
        }
        const uint32_t pid = vpn_of(dl) == dv ? pd0 : pd1;
        ds[u] = pid * PAGE_CH + (dl & (PAGE_CH - 1));
        const uint64_t slot = (cur.first + e) & (L - 1);
        const uint64_t si = (((cur.sm >> e) & 1ull) * n64 + cur.src) * L + slot;
        const uint32_t sl = s0 + ei * cur.ncu + c;
        const uint8_t* sp = ring ? p.pool + ((uint64_t)(vpn_of(sl) == sv ? ps0 : ps1) * PAGE_BYTES) + ((sl & (PAGE_CH - 1)) << 4)
                            : wire ? p.wire + cur.spos + 16ull * cur.src + 16ull * (e * cur.ncu + c)
                            : cur.kind == SRC_CMD
                                ? p.cmds + (uint64_t)cur.src * p.cmd_cap + 16ull * ((uint32_t)cur.spos + (e - cur.e0) * cur.ncu + c)
                                : p.slabs + (((uint64_t)cur.src * rows + cur.g) * p.E + e) * P + c * 16;
        sp = act ? sp : dummy;
        const uint32_t* wp = (ring && act) ? &p.info[si].x
                             : (wire && act) ? reinterpret_cast<const uint32_t*>(p.wire + cur.spos + 16ull * e + 8)
                                             : reinterpret_cast<const uint32_t*>(dummy);
#ifdef RG_BULK_NT_LOAD  // ablation: non-temporal loads (r01: 1.115 vs 1.090 ms plain)
        x[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(sp));
#else  // temporal: the second follower's read of the same leader entries hits L2 / Infinity Cache
        x[u] = *reinterpret_cast<const u32x4*>(sp);
#endif
        want[u] = *wp;
        // the slot's job, for its consume in the next pass
        sq[u] = cur.q; sdp[u] = cur.dpos;
        ss[u] = (uint32_t)((cur.first + cur.b) & (L - 1));
        sbk[u] = (Banks)(cur.dm >> (cur.b & 63u));
        sm[u] = (cur.b & 0x7Fu) | ((cur.e0 & 0x7Fu) << 7) | ((cur.ncu & 0x7Fu) << 14) |
                ((step ? min(EPI, cur.n - cur.b) : 0u) << 21) |
                ((ring || (WIRE && cur.kind == SRC_WIRE)) ? 1u << 28 : 0u);  // followers verify the sender's CRC
        vmask = step ? (vmask | (1u << u)) : (vmask & ~(1u << u));
        cur.b += step ? EPI : 0u;
      }
    }
    if (cur.live && !cur.uni && vmask == 0) {  // a non-uniform job once the ring has drained
      vjob<LG, WIRE>(p, pt, cur, crc);
      cur.b = cur.n;
    }
    if (cur.live && cur.b >= cur.n) cur.live = next_job<LG, WIRE, true>(p, cur, tj, stride, ntiles, pt);
  } while (rfl((uint32_t)(vmask != 0 || cur.live)));
  } else {
  // ring slot u: payload chunk, destination pool chunk, sender's slot CRC (per lane); the entries
  // each slot's step holds are wave-uniform: 8 bits per slot in one scalar (ikv / ckv), so the
  // per-lane flags need no registers of their own (r03: 99 -> 95 VGPRs, occupancy 4 -> 5)
  u32x4 x[BULK_U];
  uint32_t ds[BULK_U], want[BULK_U];
#pragma unroll
  for (int u = 0; u < BULK_U; ++u) {
    x[u] = u32x4{0, 0, 0, 0};
    ds[u] = want[u] = 0;
  }
  // Every slot issues exactly two loads per pass (payload chunk + sender CRC word), redirected to a
  // dummy address when the slot has no work, so the number of memory operations between a load
  // and its use is the same on every path and the compiler's vmcnt waits keep the ring in flight.
  // A pass never spans two jobs (the cursor moves once per pass), so the slots consumed in a pass
  // all belong to the job `pj` the previous pass issued.
  const uint8_t* dummy = reinterpret_cast<const uint8_t*>(p.crc_tab + CRC_ZERO_OFF);  // 16 zero bytes
  uint32_t vmask = 0;
  uint32_t iq = 0, ib = 0, ie0 = 0, idp = 0, incu = 0, ikv = 0;  // the job of the pass being issued (for its consume)
  bool ichk = false;
  uint64_t ifirst = 0, idm = 0;
  do {
    const uint32_t cq = iq, cb = ib, ce0 = ie0, cdp = idp, cncu = incu, ckv = ikv;
    const bool cchk = ichk;
    const uint64_t cfirst = ifirst, cdm = idm;
    iq = cur.q; ib = cur.b; ie0 = cur.e0; idp = cur.dpos; incu = cur.ncu; ifirst = cur.first; idm = cur.dm;
    ichk = cur.kind == SRC_RING || (WIRE && cur.kind == SRC_WIRE);  // followers verify the sender's CRC
    ikv = 0;
#ifndef RG_BULK_STEP_PT
    // the pass's page ids: its BULK_U steps are consecutive in the job, at most 64 chunks each, so the
    // pass covers at most BULK_U * 64 = PAGE_CH destination (and source) chunks: two pages each. Four
    // scalar loads per pass, issued together, instead of four per step.
    static_assert(BULK_U * 64 <= PAGE_CH, "a pass spans at most two stream pages");
    const uint32_t qdv = vpn_of(cur.dpos + (cur.b - cur.e0) * cur.ncu);
    const uint32_t qsv = vpn_of((uint32_t)cur.spos + cur.b * cur.ncu);
    uint32_t qd0 = 0, qd1 = 0, qs0 = 0, qs1 = 0;
    if (cur.live && cur.uni && cur.b < cur.n && cur.ncu) {
      const uint64_t dr = (uint64_t)cur.q * p.PTS;
      qd0 = pt[dr + (qdv & PTSM)];
      qd1 = pt[dr + ((qdv + 1) & PTSM)];
      if (cur.kind == SRC_RING) {
        const uint64_t sr = (uint64_t)cur.src * p.PTS;
        qs0 = pt[sr + (qsv & PTSM)];
        qs1 = pt[sr + ((qsv + 1) & PTSM)];
      }
    }
#endif
#pragma unroll
    for (int u = 0; u < BULK_U; ++u) {
      {  // consume slot u: store, CRC, info, verify (fl = 0 for an empty slot: no stores). A stream's
        // Cmd is followed by zeros up to its chunk boundary (every writer copies whole chunks), and
        // lanes past a Cmd's chunks contribute nothing, so the CRC is the slot CRC.
        const bool valid = ei < ((ckv >> (8 * u)) & 0xFFu);
        const bool act = valid && c < cncu;
        if (act) {
#ifdef RG_BULK_PLAIN_STORE
          *reinterpret_cast<u32x4*>(p.pool + (uint64_t)ds[u] * 16) = x[u];
#else
          __builtin_nontemporal_store(x[u], reinterpret_cast<u32x4*>(p.pool + (uint64_t)ds[u] * 16));
#endif
        }
        uint32_t v = 0;
#ifndef RG_BULK_NOCRC
        v = crc.raw16(make_uint4(x[u].x, x[u].y, x[u].z, x[u].w));
#endif
        if constexpr (LG > 0) v = xor_lanes<LG>(crc.shift(v));  // raw(slot) = XOR_c Z^(after c)(raw c)
        if (valid && c == 0) {
          const uint32_t e = cb + u * EPI + ei;
          put_info(p, cq, cfirst, cdm, e, act ? (p.crc_const ^ v) : 0u, cdp + (e - ce0) * cncu, cchk && act, want[u]);
        }
      }
      {  // issue the job's next step (or an empty step) into slot u
        const bool step = cur.live && cur.uni && cur.b < cur.n;
        const uint32_t e = cur.b + ei;
        const bool valid = step && e < cur.n;
        const bool act = valid && c < cur.ncu;
        const bool ring = cur.kind == SRC_RING, wire = WIRE && (cur.kind == SRC_WIRE || cur.kind == SRC_WIRE_PROP);
        // destination chunks of this step: at most 64, so at most two stream pages (page ids by
        // scalar loads: uniform addresses)
        const uint32_t d0 = cur.dpos + (cur.b - cur.e0) * cur.ncu;
        const uint32_t dl = d0 + ei * cur.ncu + c;
        const uint32_t s0 = (uint32_t)cur.spos + cur.b * cur.ncu;
#ifdef RG_BULK_STEP_PT  // A/B: the step's own page ids (r03h product)
        const uint32_t dv = vpn_of(d0), sv = vpn_of(s0);
        uint32_t pd0 = 0, pd1 = 0, ps0 = 0, ps1 = 0;
        if (step && cur.ncu) {
          const uint64_t dr = (uint64_t)cur.q * p.PTS;
          pd0 = pt[dr + (dv & PTSM)];
          pd1 = pt[dr + ((dv + 1) & PTSM)];
          if (ring) {
            const uint64_t sr = (uint64_t)cur.src * p.PTS;
            ps0 = pt[sr + (sv & PTSM)];
            ps1 = pt[sr + ((sv + 1) & PTSM)];
          }
        }
#else
        const uint32_t dv = qdv, sv = qsv, pd0 = qd0, pd1 = qd1, ps0 = qs0, ps1 = qs1;
#endif
        const uint32_t pid = vpn_of(dl) == dv ? pd0 : pd1;
        ds[u] = pid * PAGE_CH + (dl & (PAGE_CH - 1));
        ikv |= (step ? min(EPI, cur.n - cur.b) : 0u) << (8 * u);
        const uint64_t slot = (cur.first + e) & (L - 1);
        const uint64_t si = (((cur.sm >> e) & 1ull) * n64 + cur.src) * L + slot;
        const uint32_t sl = s0 + ei * cur.ncu + c;
        const uint8_t* sp = ring ? p.pool + ((uint64_t)(vpn_of(sl) == sv ? ps0 : ps1) * PAGE_BYTES) + ((sl & (PAGE_CH - 1)) << 4)
                            : wire ? p.wire + cur.spos + 16ull * cur.src + 16ull * (e * cur.ncu + c)
                            : cur.kind == SRC_CMD
                                ? p.cmds + (uint64_t)cur.src * p.cmd_cap + 16ull * ((uint32_t)cur.spos + (e - cur.e0) * cur.ncu + c)
                                : p.slabs + (((uint64_t)cur.src * rows + cur.g) * p.E + e) * P + c * 16;
        sp = act ? sp : dummy;
        const uint32_t* wp = (ring && act) ? &p.info[si].x
                             : (wire && act) ? reinterpret_cast<const uint32_t*>(p.wire + cur.spos + 16ull * e + 8)
                                             : reinterpret_cast<const uint32_t*>(dummy);
#ifdef RG_BULK_NT_LOAD  // ablation: non-temporal loads (r01: 1.115 vs 1.090 ms plain)
        x[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(sp));
#else  // temporal: the second follower's read of the same leader entries hits L2 / Infinity Cache
        x[u] = *reinterpret_cast<const u32x4*>(sp);
#endif
        want[u] = *wp;
        vmask = step ? (vmask | (1u << u)) : (vmask & ~(1u << u));
        cur.b += step ? EPI : 0u;
      }
    }
    if (cur.live && !cur.uni && vmask == 0) {  // a non-uniform job once the ring has drained
      vjob<LG, WIRE>(p, pt, cur, crc);
      cur.b = cur.n;
    }
    if (cur.live && cur.b >= cur.n) cur.live = next_job<LG, WIRE>(p, cur, tj, stride, ntiles);
  } while (rfl((uint32_t)(vmask != 0 || cur.live)));
  }
}

static int lg_of(uint32_t P) {
  int lg = 0;
  while ((16u << lg) < P) ++lg;
  return lg;
}

int bulk_lds_bytes(uint32_t P) {
  return P ? (int)((CRC_T_WORDS + CRC_N_WORDS + (P / 16) * CRC_SH_STRIDE + CRC_ZP_WORDS) * 4) : 16;
}

template <bool W, bool MJ, class F>
static hipError_t with_bulk_w(uint32_t P, F f) {
#ifdef RG_DEV_ONLY_LG  // development builds: one payload size only (ISA / resource checks)
  if (W || MJ || lg_of(P) != RG_DEV_ONLY_LG) return hipErrorInvalidValue;
  return f(bulk_kernel<RG_DEV_ONLY_LG, false, false>);
#endif
  switch (lg_of(P)) {
    case 0: return f(bulk_kernel<0, W, MJ>);
    case 1: return f(bulk_kernel<1, W, MJ>);
    case 2: return f(bulk_kernel<2, W, MJ>);
    case 3: return f(bulk_kernel<3, W, MJ>);
    case 4: return f(bulk_kernel<4, W, MJ>);
    case 5: return f(bulk_kernel<5, W, MJ>);
    case 6: return f(bulk_kernel<6, W, MJ>);
    default: return hipErrorInvalidValue;
  }
}
template <class F>
static hipError_t with_bulk(uint32_t P, bool wire, bool mj, F f) {
  if (!P) return hipSuccess;  // metadata-only engines have no payload stage (tick_impl)
  if (mj) return wire ? with_bulk_w<true, true>(P, f) : with_bulk_w<false, true>(P, f);
  return wire ? with_bulk_w<true, false>(P, f) : with_bulk_w<false, false>(P, f);
}

int bulk_blocks_per_cu(uint32_t P) {
  int n = 0;
  const hipError_t r = with_bulk(P, false, false, [&](auto k) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 256, bulk_lds_bytes(P));
  });
  return (r == hipSuccess && n > 0) ? n : 1;
}

hipError_t launch_bulk(const BulkParams& p, const uint32_t* pt, hipStream_t s, int grid) {
  return with_bulk(p.P, p.wire_mode != 0, p.multijob != 0, [&](auto k) {
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), bulk_lds_bytes(p.P), s, p, pt);
    return hipGetLastError();
  });
}

// ================================================================== payload page pool
// One lane per replica (coalesced state rows): return the stream pages control released
// ([S_LPG, S_NLPG)) to the free ring and take the pages this step's appends need ([S_APG,
// ceil(S_HW))). The ring positions come from a block-wide scan and ONE tail and ONE head atomic
// per 1,024-lane block (r03: an atomic pair per wave, 3,072 pairs on two addresses at 64K x 3, made
// this a 55 µs kernel). Allocations read ids below `limit` (written by an earlier launch); frees
// write at and above the tail: disjoint.
constexpr uint32_t POOL_BLOCK = 1024;
__global__ void __launch_bounds__(POOL_BLOCK) pool_kernel(PoolParams pp) {
  __shared__ uint32_t wf[POOL_BLOCK / 64], wa[POOL_BLOCK / 64];
  __shared__ unsigned long long base[2];
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x, lane = lane_id(), w = threadIdx.x >> 6;
  const bool valid = q < pp.nrep;
  const uint64_t n = pp.nrep, PTSM = pp.PTS - 1;
  uint32_t lpg = 0, apg = 0, nlpg = 0, top = 0, f = 0, a = 0;
  if (valid) {
    lpg = pp.s32_in[S_LPG * n + q];
    apg = pp.s32_in[S_APG * n + q];
    nlpg = pp.s32_out[S_NLPG * n + q];
    top = vpn_ceil(pp.s32_out[S_HW * n + q]);
    f = vpn_diff(nlpg, lpg);
    a = vpn_diff(top, apg);
  }
  uint32_t fo = wave_excl_scan32(f), ao = wave_excl_scan32(a);
  if (lane == 63) {
    wf[w] = fo + f;
    wa[w] = ao + a;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // the block's wave totals → offsets, and the block's two ring reservations
    uint32_t sf = 0, sa = 0;
    for (uint32_t i = 0; i < blockDim.x / 64; ++i) {
      const uint32_t tf = wf[i], ta = wa[i];
      wf[i] = sf;
      wa[i] = sa;
      sf += tf;
      sa += ta;
    }
    base[0] = sf ? atomicAdd(&pp.ctl->tail, (unsigned long long)sf) : 0ull;
    base[1] = sa ? atomicAdd(&pp.ctl->head, (unsigned long long)sa) : 0ull;
  }
  __syncthreads();
  const unsigned long long fb = base[0] + wf[w], ab = base[1] + wa[w];
  const unsigned long long limit = pp.ctl->limit;
  uint32_t* ptq = pp.pt + (uint64_t)q * pp.PTS;
  for (uint32_t k = 0; k < f; k += 8) {  // frees: eight page-table reads in flight, then their ring writes
    uint32_t v[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) v[j] = k + j < f ? ptq[(lpg + k + j) & PTSM] : 0u;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j)
      if (k + j < f) pp.fring[(fb + fo + k + j) % pp.npages] = v[j];
  }
  const bool ok = ab + ao + a <= limit;
  if (ok) {
    for (uint32_t k = 0; k < a; k += 8) {
      uint32_t v[8];
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) v[j] = k + j < a ? pp.fring[(ab + ao + k + j) % pp.npages] : 0u;
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j)
        if (k + j < a) ptq[(apg + k + j) & PTSM] = v[j];
    }
  }
  if (valid) {
    pp.s32_out[S_LPG * n + q] = nlpg;
    pp.s32_out[S_APG * n + q] = ok ? top : apg;
    if (!ok) {  // the pool is empty: this replica's appends of the step are not stored; the engine is poisoned
      pp.s32_out[S_ERR * n + q] |= ERR_POOL;
      pp.jcnt[q] = 0;
      atomicOr(&pp.ctl->fail, 1u);
    }
  }
}

hipError_t launch_pool(const PoolParams& p, hipStream_t s) {
  hipLaunchKernelGGL(pool_kernel, dim3((p.nrep + POOL_BLOCK - 1) / POOL_BLOCK), dim3(POOL_BLOCK), 0, s, p);
  return hipGetLastError();
}

__global__ void pool_reset_kernel(uint32_t* fring, uint64_t npages, PoolCtl* ctl) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < npages; i += (uint64_t)gridDim.x * blockDim.x)
    fring[i] = (uint32_t)i;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ctl->head = 0;
    ctl->tail = ctl->limit = npages;
    ctl->fail = 0;
    ctl->param_err = 0;
  }
}

hipError_t launch_pool_reset(uint32_t* fring, uint64_t npages, PoolCtl* ctl, hipStream_t s) {
  hipLaunchKernelGGL(pool_reset_kernel, dim3(1024), dim3(256), 0, s, fring, npages, ctl);
  return hipGetLastError();
}

// ================================================================== bootstrap (peer.go Launch + bootstrap)
// A new replica (join = false): becomeFollower(1), then one ConfigChange entry per slot at term 1,
// indices 1..R — AddNode(s) for each initial member s (descriptor 0 for the others), committed R,
// and its remotes as addNode set them. A joining replica (rg_config.join_slots, StartOnDiskReplica
// with join = true): becomeFollower(0) with an empty log and no membership; it learns the
// membership from the log or a snapshot its leader sends once a ConfigChange adds it.
__global__ void bootstrap_kernel(TickParams p, uint2* info) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= p.nrep) return;
  const uint32_t R = p.R, s = q / p.G, g = q - s * p.G;
  const uint64_t n = p.nrep;
  const bool joining = (p.JS >> s) & 1u;
  uint64_t* a = p.s64_out + q;
  for (uint32_t f = 0; f < S64_ROWS; ++f) a[f * n] = 0;
  uint32_t* b = p.s32_out + q;
  for (uint32_t f = 0; f < S32_ROWS; ++f) b[f * n] = 0;
  const uint32_t im = (p.IM ? p.IM : (1u << R) - 1u) & ~p.JS;  // initialMembers
  const uint64_t last = joining ? 0 : R;
  a[S_TERM * n] = joining ? 0 : 1;  // becomeFollower(term, NoLeader): one reset
  a[S_LAST * n] = last;
  a[S_COMMITTED * n] = last;
  a[S_CC_HI * n] = last;
  b[S_RNG_CTR * n] = 1;
  b[S_MEMBERS * n] = joining ? 0u : im;
  b[S_SNAP_MEMBERS * n] = joining ? 0u : im;
  const uint64_t key = (pl_group(p.pl, s, g) << 32) | ((uint64_t)s << 24) | 1ull;
  b[S_RAND_TO * n] = p.ET + (uint32_t)(mix64(p.seed ^ mix64(key)) % p.ET);
  for (uint32_t j = 0; j < R; ++j) {  // addNode → setRemote(id, 0, last+1)
    p.rem_out[(0 * R + j) * n + q] = 0;
    p.rem_out[(1 * R + j) * n + q] = last + 1;
    p.rem_out[(2 * R + j) * n + q] = 0;
    p.rst_out[j * n + q] = RETRY;
  }
  for (uint32_t i = 1; i <= last; ++i) {
    const uint64_t slot = i & (p.L - 1);
    const uint32_t cc = ((im >> (i - 1)) & 1u) ? (CC_ADD << 4 | i) : 0u;  // AddNode(slot i - 1)
    p.tr[slot * n + q] = 1ull | TYPE_BIT | cc_bits(cc);  // ConfigChange, term 1, no payload, bank 0
    info[(uint64_t)q * p.L + slot] = make_uint2(0u, 0u);  // no Cmd bytes, at stream position 0
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
    if (wi == 0) slab_info[at / wpe] = make_uint2(SYN_OFF, P);  // a generator Cmd: P bytes at its slab slot
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
// The Cmd bytes themselves reach their slab's arena with one H2D copy (the host lays them out
// chunk-aligned and zero-padded in pinned staging); this scatters their slab_info descriptors.
__global__ void stage_cmds_kernel(StageParams a) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * blockDim.x)
    a.slab_info[a.info_at[i]] = make_uint2(a.chunk[i], a.len[i]);
}

hipError_t launch_stage_cmds(const StageParams& a, hipStream_t s) {
  if (!a.n) return hipSuccess;
  const uint64_t blocks = std::min<uint64_t>((a.n + 255) / 256, 4096);
  hipLaunchKernelGGL(stage_cmds_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, a);
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

// ================================================================== copy-back to host-mapped memory
// rg_apply_async's PCIe leg: a few workgroups stream the gathered batch from device staging into
// pinned host memory, four 16-B chunks in flight per lane (the tail, under 16 B, by single bytes)
__global__ void __launch_bounds__(256) copy_to_host_kernel(const uint8_t* src, uint8_t* dst, uint64_t bytes) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint64_t n = bytes / 16, stride = (uint64_t)gridDim.x * 256 * 4;
  for (uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x; i < n; i += stride) {
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      v[k] = i + 256 * k < n ? *reinterpret_cast<const u32x4*>(src + (i + 256 * k) * 16) : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (i + 256 * k < n) __builtin_nontemporal_store(v[k], reinterpret_cast<u32x4*>(dst + (i + 256 * k) * 16));
  }
  if (blockIdx.x == 0 && threadIdx.x < (bytes & 15)) dst[n * 16 + threadIdx.x] = src[n * 16 + threadIdx.x];
}

hipError_t launch_copy_to_host(const void* src, void* dst, uint64_t bytes, hipStream_t s) {
  if (!bytes) return hipSuccess;
  static const int blocks = [] {
    const char* v = getenv("RAFTGPU_COPY_WG");  // measurement override
    return v && atoi(v) > 0 ? atoi(v) : 32;
  }();
  hipLaunchKernelGGL(copy_to_host_kernel, dim3(blocks), dim3(256), 0, s, (const uint8_t*)src, (uint8_t*)dst, bytes);
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
