// raftgpu_kernels.hip — the MI355X Raft tick: a control kernel (all Raft logic, one lane per
// replica; raftgpu_ctl.hip) followed by a bulk kernel (entry payload copy + CRC-32;
// raftgpu_bulk.hip). This unit holds their dispatchers and the small kernels around them (page
// pool, bootstrap, payload generator, staging, probes, reductions).
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
#include "raftgpu_dev.h"

namespace rg {

hipError_t launch_control(const TickParams* p, uint32_t* perr, uint32_t R, uint32_t nrep, hipStream_t s) {
  switch (R) {
    case 1: return launch_control_t<1>(p, perr, nrep, s);
    case 2: return launch_control_t<2>(p, perr, nrep, s);
    case 3: return launch_control_t<3>(p, perr, nrep, s);
    case 4: return launch_control_t<4>(p, perr, nrep, s);
    case 5: return launch_control_t<5>(p, perr, nrep, s);
    case 6: return launch_control_t<6>(p, perr, nrep, s);
    case 7: return launch_control_t<7>(p, perr, nrep, s);
    case 8: return launch_control_t<8>(p, perr, nrep, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_control_fast(const TickParams* p, uint32_t* perr, uint32_t R, uint32_t nrep, bool fb, hipStream_t s) {
  switch (R) {
    case 1: return launch_control_fast_t<1>(p, perr, nrep, fb, s);
    case 2: return launch_control_fast_t<2>(p, perr, nrep, fb, s);
    case 3: return launch_control_fast_t<3>(p, perr, nrep, fb, s);
    case 4: return launch_control_fast_t<4>(p, perr, nrep, fb, s);
    case 5: return launch_control_fast_t<5>(p, perr, nrep, fb, s);
    case 6: return launch_control_fast_t<6>(p, perr, nrep, fb, s);
    case 7: return launch_control_fast_t<7>(p, perr, nrep, fb, s);
    case 8: return launch_control_fast_t<8>(p, perr, nrep, fb, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_control_resident(const TickParams* p, uint32_t k, uint32_t* perr, uint32_t R, uint32_t G,
                                   hipStream_t s) {
  switch (R) {
    case 1: return launch_control_resident_t<1>(p, k, perr, G, s);
    case 2: return launch_control_resident_t<2>(p, k, perr, G, s);
    case 3: return launch_control_resident_t<3>(p, k, perr, G, s);
    case 4: return launch_control_resident_t<4>(p, k, perr, G, s);
    default: return hipErrorInvalidValue;  // R > 4: a control wave needs a SIMD of its own
  }
}

int bulk_lds_bytes(uint32_t P) {
  return P ? (int)((CRC_T_WORDS + CRC_N_WORDS + (P / 16) * CRC_SH_STRIDE + CRC_ZP_WORDS) * 4) : 16;
}

int bulk_blocks_per_cu(uint32_t P) { return P ? bulk_occupancy_t<false, false>(P) : 1; }

hipError_t launch_bulk(const BulkParams& p, const uint32_t* pt, hipStream_t s, int grid) {
  if (!p.P) return hipSuccess;  // metadata-only engines have no payload stage (tick_impl)
  if (p.multijob) return p.wire_mode ? launch_bulk_t<true, true>(p, pt, s, grid) : launch_bulk_t<false, true>(p, pt, s, grid);
  return p.wire_mode ? launch_bulk_t<true, false>(p, pt, s, grid) : launch_bulk_t<false, false>(p, pt, s, grid);
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
  // a control launch of this tick (or an earlier one) skipped a corrupt parameter block: its state rows
  // and job counts are stale, so nothing is freed or allocated (the engine is poisoned, rg_sync reports it)
  if (pp.ctl->param_err) return;
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x, lane = lane_id(), w = threadIdx.x >> 6;
  const bool valid = q < pp.nrep;
  // ids below limit were published by an earlier launch (bulk_kernel) and do not change in this one:
  // loaded with the state rows, not after the block's reservations (one round trip fewer)
  const unsigned long long limit = pp.ctl->limit;
  const uint64_t n = pp.nrep, PTSM = pp.PTS - 1;
  uint32_t lpg = 0, apg = 0, nlpg = 0, top = 0, f = 0, a = 0;
  if (valid) {
    lpg = pp.s32[S_LPG * n + q];
    apg = pp.s32[S_APG * n + q];
    nlpg = pp.s32[S_NLPG * n + q];
    top = vpn_ceil(pp.s32[S_HW * n + q]);
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
  const bool ok = ab + ao + a <= limit;
  // Frees and takes are done by the whole wave, 64 consecutive page-table entries / ring slots per
  // instruction. Lane by lane, a compaction tick's frees (64 pages per replica) touched 64 cache lines
  // per instruction and took 100 µs instead of 17 (r04).
  const uint32_t AW = (uint32_t)__builtin_amdgcn_readlane((int)(ao + a), 63);
  const uint32_t qb = q - lane;
  auto owner = [&](uint32_t incl, uint32_t i) {  // the first lane whose inclusive scan exceeds i
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t step = 32; step; step >>= 1) {
      const uint32_t v = (uint32_t)__shfl((int)incl, (int)(lo + step - 1), 64);
      if (v <= i) lo += step;
    }
    return lo < 63 ? lo : 63u;
  };
  // frees: replica by replica (a compaction frees tens of pages per replica): the wave copies one
  // replica's page-table range per chunk of 64, eight chunks in flight (wave-uniform chunk list)
  {
    uint64_t m = __ballot(f != 0);
    uint32_t curL = 64, curk = 0, curf = 0;
    auto adv = [&]() -> bool {
      if (curL < 64 && curk + 64 < curf) {
        curk += 64;
        return true;
      }
      if (!m) {
        curL = 64;
        return false;
      }
      curL = (uint32_t)__ffsll((long long)m) - 1;
      m &= m - 1;
      curk = 0;
      curf = (uint32_t)__builtin_amdgcn_readlane((int)f, (int)curL);
      return true;
    };
    for (;;) {
      uint32_t cl[8], ck[8];
      uint32_t nb = 0;
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) {
        const bool has = adv();
        cl[j] = has ? curL : 64u;
        ck[j] = curk;
        nb += has ? 1u : 0u;
      }
      if (nb == 0) break;
      uint32_t v[8];
      uint64_t dst[8];
      bool act[8];
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t L = cl[j] & 63u;
        const uint32_t fL = (uint32_t)__builtin_amdgcn_readlane((int)f, (int)L);
        const uint32_t lpgL = (uint32_t)__builtin_amdgcn_readlane((int)lpg, (int)L);
        const uint32_t foL = (uint32_t)__builtin_amdgcn_readlane((int)fo, (int)L);
        const uint32_t k = ck[j] + lane;
        act[j] = cl[j] < 64 && k < fL;
        v[j] = act[j] ? pp.pt[(uint64_t)(qb + L) * pp.PTS + ((lpgL + k) & PTSM)] : 0u;
        const uint64_t b0 = (fb + foL + ck[j]) % pp.npages;  // wave-uniform: one division per chunk
        dst[j] = b0 + lane >= pp.npages ? b0 + lane - pp.npages : b0 + lane;
      }
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j)
        if (act[j]) pp.fring[dst[j]] = v[j];
    }
  }
  for (uint32_t i0 = 0; i0 < AW; i0 += 64 * 4) {  // four ring reads in flight, then their page-table writes
    uint32_t v[4], row[4], slot[4];
    bool tk[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t i = i0 + 64 * j + lane, lo = owner(ao + a, i);
      const uint32_t lao = (uint32_t)__shfl((int)ao, (int)lo, 64), lapg = (uint32_t)__shfl((int)apg, (int)lo, 64);
      const bool lok = __shfl((int)ok, (int)lo, 64) != 0;
      tk[j] = i < AW && lok;
      row[j] = qb + lo;
      slot[j] = (lapg + i - lao) & PTSM;
      v[j] = tk[j] ? pp.fring[(ab + i) % pp.npages] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
      if (tk[j]) pp.pt[(uint64_t)row[j] * pp.PTS + slot[j]] = v[j];
  }
  if (valid) {  // in place: only what moved (a replica takes a page per 16 entries of 256 B)
    if (nlpg != lpg) pp.s32[S_LPG * n + q] = nlpg;
    if ((ok ? top : apg) != apg) pp.s32[S_APG * n + q] = ok ? top : apg;
    if (!ok) {  // the pool is empty: this replica's appends of the step are not stored; the engine is poisoned
      pp.s32[S_ERR * n + q] |= ERR_POOL;
      pp.jcnt[q] = 0;
      atomicOr(&pp.ctl->fail, 1u);
    }
  }
}

hipError_t launch_pool(const PoolParams& p, hipStream_t s) {
  hipLaunchKernelGGL(pool_kernel, dim3((p.nrep + POOL_BLOCK - 1) / POOL_BLOCK), dim3(POOL_BLOCK), 0, s, p);
  return hipGetLastError();
}

__global__ void pool_reset_kernel(uint32_t* fring, uint64_t npages, PoolCtl* ctl, uint64_t mul) {
  // the ring starts as the permutation i -> i * mul mod npages (mul coprime to npages)
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < npages; i += (uint64_t)gridDim.x * blockDim.x)
    fring[i] = (uint32_t)(mul > 1 ? (i * mul) % npages : i);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ctl->head = 0;
    ctl->tail = ctl->limit = npages;
    ctl->fail = 0;
    ctl->param_err = 0;
  }
}

hipError_t launch_pool_reset(uint32_t* fring, uint64_t npages, PoolCtl* ctl, hipStream_t s) {
  // The ring starts as the permutation i -> i * 1000003 mod npages (a prime multiplier: a bijection
  // unless it divides npages), so the pages consecutive replicas take lie ~4 GB apart instead of side
  // by side: the first snapshot window's payload stage ran 3 % faster so (r04v, per-tick kernel
  // trace; r04 A/B: 65,537 ties, 4,099 and 257 lose 2-3 %; -DRG_AB_POOL_PERM=<m> builds another).
  uint64_t mul = npages % 1000003ull ? 1000003ull : 1000033ull;
#ifdef RG_AB_POOL_PERM
  mul = RG_AB_POOL_PERM;
#endif
  {
    uint64_t a = mul, b = npages;
    while (b) {
      const uint64_t t = a % b;
      a = b;
      b = t;
    }
    if (mul == 0 || a != 1) mul = 1;  // not coprime: the identity
  }
  hipLaunchKernelGGL(pool_reset_kernel, dim3(1024), dim3(256), 0, s, fring, npages, ctl, mul);
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
  uint64_t* a = p.s64 + q;
  for (uint32_t f = 0; f < S64_ROWS; ++f) a[f * n] = 0;
  uint32_t* b = p.s32 + q;
  for (uint32_t f = 0; f < S32_ROWS; ++f) b[f * n] = 0;
  const uint32_t im = (p.IM ? p.IM : (1u << R) - 1u) & ~p.JS;  // initialMembers
  const uint64_t last = joining ? 0 : R;
  a[S_TERM * n] = joining ? 0 : 1;  // becomeFollower(term, NoLeader): one reset
  a[S_LAST * n] = last;
  a[S_LAST_TERM * n] = last ? 1 : 0;  // the bootstrap entries are at term 1
  a[S_COMMITTED * n] = last;
  a[S_CC_HI * n] = last;
  b[S_RNG_CTR * n] = 1;
  b[S_MEMBERS * n] = joining ? 0u : im;
  b[S_SNAP_MEMBERS * n] = joining ? 0u : im;
  const uint64_t key = (pl_group(p.pl, s, g) << 32) | ((uint64_t)s << 24) | 1ull;
  b[S_RAND_TO * n] = p.ET + (uint32_t)(mix64(p.seed ^ mix64(key)) % p.ET);
  for (uint32_t j = 0; j < R; ++j) {  // addNode → setRemote(id, 0, last+1)
    p.rem[(0 * R + j) * n + q] = 0;
    p.rem[(1 * R + j) * n + q] = last + 1;
    p.rem[(2 * R + j) * n + q] = 0;
    p.rst[j * n + q] = RETRY;
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
// a wave per batch: lane x writes Cmd x's {arena chunk, len} descriptor (chunks by a wave scan of the
// chunk counts) and zeroes the bytes between its end and its last chunk's end (the slot CRC reads them)
__global__ void __launch_bounds__(256) stage_cmds_kernel(StageParams a) {
  const uint64_t b = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= a.n) return;
  const uint32_t x = threadIdx.x & 63u, cnt = a.count[b];
  const uint32_t len = x < cnt ? a.lens[a.first[b] + x] : 0u, nc = (len + 15u) >> 4;
  const uint32_t chunk = a.chunk[b] + wave_excl_scan32(nc);
  if (x >= cnt) return;
  a.slab_info[a.info_at[b] + x] = make_uint2(chunk, len);
  if (len & 15u) {
    uint8_t* t = a.arena + (uint64_t)chunk * 16 + len;
    for (uint32_t k = len & 15u; k < 16u; ++k) *t++ = 0;
  }
}

hipError_t launch_stage_cmds(const StageParams& a, hipStream_t s) {
  if (!a.n) return hipSuccess;
  hipLaunchKernelGGL(stage_cmds_kernel, dim3((uint32_t)((a.n + 3) / 4)), dim3(256), 0, s, a);
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
#ifdef RG_AB_COPY_WG  // A/B variant (r03: 2-16 workgroups lost to 32)
  constexpr int blocks = RG_AB_COPY_WG;
#else
  constexpr int blocks = 32;
#endif
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

// Σ_g max_s committed, on the state a next tick would read (s64). With ranks > 1 the replicas
// of a column belong to different groups: sum the slot-0 replicas hosted here (each group's slot 0
// lives on exactly one rank, so the sum over ranks counts every group once).
__global__ void sum_committed_kernel(TickParams p, unsigned long long* out) {
  uint64_t acc = 0;
  const uint32_t ns = p.pl.N > 1 ? 1u : p.R;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < p.G; g += gridDim.x * blockDim.x) {
    uint64_t m = 0;
    for (uint32_t s = 0; s < ns; ++s) m = umax64(m, p.s64[(uint64_t)S_COMMITTED * p.nrep + (uint64_t)s * p.G + g]);
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
// p is the parameter block a next tick would use (s64 = current state, cnt_in/hdr_in = the last
// tick's outbox) with job32 / jcnt pointed at the last tick's copy jobs: a replica's appended
// entries are its jobs' entry counts (what the bulk kernel moved for it).
__global__ void traffic_kernel(TickParams p, unsigned long long* out6) {
  uint64_t v[5] = {0, 0, 0, 0, 0};
  const uint64_t n = p.nrep, JN = (uint64_t)p.J * n;
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < p.nrep; q += gridDim.x * blockDim.x) {
    const uint32_t s = q / p.G, g = q - s * p.G;
    const bool ld = p.s32[S_ROLE * n + q] == LEADER;
    v[0] += ld;
    for (uint32_t d = 0; d < p.R; ++d) {
      const uint32_t c = cnt_n(p.cnt_in[((uint64_t)s * p.R + d) * p.G + g]);
      v[1] += c;
      for (uint32_t k = 0; k < c; ++k) {
        const uint64_t w0 = p.hdr_in[(((uint64_t)s * p.R + d) * p.K + k) * p.G + g];
        if ((w0 & 0xFF) == M_REPLICATE) v[2] += w0 >> 32;
      }
    }
    uint64_t app = 0;
    const uint32_t nj = p.jcnt[q] < p.J ? p.jcnt[q] : p.J;
    for (uint32_t j = 0; j < nj; ++j) {
      const uint32_t m = p.job32[J_META * JN + (uint64_t)j * n + q];
      app += (m & 0xFF) - ((m >> 8) & 0xFF);
    }
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
