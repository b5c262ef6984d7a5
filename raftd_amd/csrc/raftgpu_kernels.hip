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
#include "raftgpu_control.h"

namespace rg {

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

template <int R>
__global__ void __launch_bounds__(256) control_kernel(TickParams p) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= p.nrep) return;
  Ctl<R> c(p, q);
  c.run();
}

hipError_t launch_control(const TickParams& p, hipStream_t s) {
  dim3 grid((p.nrep + 255) / 256), block(256);
  switch (p.R) {
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
  const uint32_t* T;  // LDS [16][256]
  const uint32_t* S;  // LDS [lg][4][256]
  __device__ __forceinline__ uint32_t raw16(uint4 v) const {
    uint32_t r = 0;
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int qd = 0; qd < 4; ++qd)
#pragma unroll
      for (int j = 0; j < 4; ++j) r ^= T[(15 - (4 * qd + j)) * 256 + ((d[qd] >> (8 * j)) & 0xFF)];
    return r;
  }
  __device__ __forceinline__ uint32_t shift(uint32_t v, int lvl) const {
    const uint32_t* sh = S + lvl * 1024;
    return sh[v & 0xFF] ^ sh[256 + ((v >> 8) & 0xFF)] ^ sh[512 + ((v >> 16) & 0xFF)] ^ sh[768 + (v >> 24)];
  }
};

#ifndef RG_BULK_U
#define RG_BULK_U 8
#endif
constexpr int BULK_U = RG_BULK_U;  // 16-B chunks in flight per lane

// One copy job, its fields uniform across the wave (SGPRs): n entries from `first`, payloads
// from the sender's ring or a proposal slab into this replica's ring, CRC per entry.
struct Job {
  uint64_t first, dm, sm, hm, tm;
  uint32_t meta, src;
};

__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t l) {
  return ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l) << 32) | __builtin_amdgcn_readlane((uint32_t)v, l);
}

__device__ __forceinline__ bool bulk_job(const BulkParams& p, const Crc& crc, uint32_t q, const Job& jb) {
  const uint64_t n64 = p.nrep;
  const uint64_t first = jb.first, dm = jb.dm, sm = jb.sm, hm = jb.hm, tm = jb.tm;
  const uint32_t n = jb.meta & 0xFF, e0 = (jb.meta >> 8) & 0xFF, kind = jb.meta >> 16, src = jb.src;
  const uint32_t lane = lane_id();
  const uint64_t L = p.L, P = p.P;
  if (P == 0) {
    const uint32_t e = lane;
    if (e >= e0 && e < n) {
      const uint64_t slot = (first + e) & (L - 1);
      const uint32_t db = (uint32_t)(dm >> e) & 1u;
      p.info[((uint64_t)db * n64 + q) * L + slot] = make_uint2(0u, (uint32_t)((tm >> e) & 1u) << 24);
    }
    return false;
  }
  const uint32_t lg = 31 - __clz((uint32_t)(P >> 4));
  const uint32_t nch = 1u << lg, epi = 64u >> lg;
  const uint32_t c = lane & (nch - 1), ei = lane >> lg;
  const uint32_t g = q % p.G;
  bool bad = false;
  for (uint32_t b = e0; b < n; b += epi * BULK_U) {
    // issue phase: every payload chunk of the batch and, for followers, the sender's stored CRC
    uint4 x[BULK_U];
    uint32_t want[BULK_U];
#pragma unroll
    for (int u = 0; u < BULK_U; ++u) {
      const uint32_t e = b + u * epi + ei;
      x[u] = make_uint4(0, 0, 0, 0);
      want[u] = 0;
      if (e < n && ((hm >> e) & 1ull)) {
        const uint64_t slot = (first + e) & (L - 1);
        const uint8_t* sp;
        if (kind == SRC_RING) {
          const uint64_t sb = (sm >> e) & 1ull;
          sp = p.pay + ((sb * n64 + src) * L + slot) * P + c * 16;
          if (c == 0) want[u] = p.info[(sb * n64 + src) * L + slot].x;
        } else {
          sp = p.slabs + (((uint64_t)src * p.G + g) * p.E + e) * P + c * 16;
        }
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 xv = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(sp));
        x[u] = make_uint4(xv.x, xv.y, xv.z, xv.w);
      }
    }
    // consume phase: store, CRC, info, verify
#pragma unroll
    for (int u = 0; u < BULK_U; ++u) {
      const uint32_t e = b + u * epi + ei;
      const bool valid = e < n;
      const bool act = valid && ((hm >> e) & 1ull);
      const uint64_t slot = (first + e) & (L - 1);
      const uint32_t db = valid ? (uint32_t)(dm >> e) & 1u : 0u;
      uint32_t v = 0;
      if (act) {
        typedef uint32_t u32x4s __attribute__((ext_vector_type(4)));
        u32x4s xs = {x[u].x, x[u].y, x[u].z, x[u].w};
#ifdef RG_BULK_PLAIN_STORE
        *reinterpret_cast<u32x4s*>(p.pay + (((uint64_t)db * n64 + q) * L + slot) * P + c * 16) = xs;
#else
        __builtin_nontemporal_store(xs, reinterpret_cast<u32x4s*>(p.pay + (((uint64_t)db * n64 + q) * L + slot) * P + c * 16));
#endif
#ifndef RG_BULK_NOCRC
        v = crc.raw16(x[u]);
#endif
      }
      for (uint32_t l = 0; l < lg; ++l) {  // raw(A||B) = Z^|B|(raw A) ^ raw B
        const uint32_t d = 1u << l;
        const uint32_t partner = (uint32_t)__shfl_down((int)v, d, 64);
        if ((c & ((d << 1) - 1)) == 0) v = crc.shift(v, (int)l) ^ partner;
      }
      if (valid && c == 0) {
        const uint32_t cr = act ? (p.crc_const ^ v) : 0u;
        const uint32_t tl = ((uint32_t)((tm >> e) & 1u) << 24) | (act ? (uint32_t)P : 0u);
        p.info[((uint64_t)db * n64 + q) * L + slot] = make_uint2(cr, tl);
        if (kind == SRC_RING && act) bad |= want[u] != cr;
      }
    }
  }
  return bad;
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

// Each wave owns tiles of p.tile consecutive replicas. Lane i of the tile loads replica i's job
// count and first job descriptor in one round trip; the wave then runs the tile's jobs back to
// back with the fields broadcast by readlane, so only the payload loads are on the critical path.
__global__ void __launch_bounds__(256) bulk_kernel(BulkParams p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  if (p.P) {
    const uint32_t lg = 31 - __clz(p.P >> 4);
    const uint32_t words = CRC_T_WORDS + lg * 1024;
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) lds[i] = p.crc_tab[i];
  }
  __syncthreads();
  const Crc crc{lds, lds + CRC_T_WORDS};
  const uint32_t waves = blockDim.x >> 6, lane = lane_id();
  const uint32_t stride = gridDim.x * waves, T = p.tile;
  const uint32_t ntiles = (p.nrep + T - 1) / T;
  for (uint32_t t = rfl(blockIdx.x * waves + (threadIdx.x >> 6)); t < ntiles; t += stride) {
    const uint32_t q = t * T + lane;
    const bool mine = lane < T && q < p.nrep;
    const uint32_t nj = mine ? p.jcnt[q] : 0u;
    Job j0{};
    if (nj) j0 = load_job(p, q, 0);
    uint64_t m = __ballot(nj != 0);
    while (m) {
      const uint32_t l = rfl((uint32_t)__ffsll((long long)m) - 1);
      m &= m - 1;
      const uint32_t qq = t * T + l, njl = __builtin_amdgcn_readlane(nj, l);
      Job jb;
      jb.first = rl64(j0.first, l); jb.dm = rl64(j0.dm, l); jb.sm = rl64(j0.sm, l);
      jb.hm = rl64(j0.hm, l); jb.tm = rl64(j0.tm, l);
      jb.meta = __builtin_amdgcn_readlane(j0.meta, l); jb.src = __builtin_amdgcn_readlane(j0.src, l);
      bool bad = bulk_job(p, crc, qq, jb);
      for (uint32_t j = 1; j < njl; ++j) bad |= bulk_job(p, crc, qq, load_job(p, qq, j));
      if (__ballot(bad) && lane == 0) atomicOr(p.crc_err + qq, ERR_CRC);
    }
  }
}

int bulk_lds_bytes(uint32_t P) {
  if (!P) return 16;
  uint32_t lg = 0;
  while ((1u << lg) < (P >> 4)) ++lg;
  return (int)((CRC_T_WORDS + lg * 1024) * 4);
}

int bulk_blocks_per_cu(uint32_t P) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, bulk_kernel, 256, bulk_lds_bytes(P)) != hipSuccess) n = 4;
  return n > 0 ? n : 1;
}

hipError_t launch_bulk(const BulkParams& p, hipStream_t s, int grid) {
  hipLaunchKernelGGL(bulk_kernel, dim3(grid), dim3(256), bulk_lds_bytes(p.P), s, p);
  return hipGetLastError();
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
  const uint64_t key = ((uint64_t)g << 32) | ((uint64_t)s << 24) | 1ull;
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
__global__ void fill_slabs_kernel(uint8_t* slabs, uint32_t nslab, uint32_t G, uint32_t E, uint32_t P, uint64_t seed) {
  const uint64_t wpe = P / 8;
  const uint64_t total = (uint64_t)nslab * G * E * wpe;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < total; w += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t ent = w / wpe, wi = w - ent * wpe;
    const uint32_t i = (uint32_t)(ent % E);
    const uint64_t sg = ent / E;
    const uint32_t gg = (uint32_t)(sg % G), sl = (uint32_t)(sg / G);
    const uint64_t key = mix64(((uint64_t)sl << 56) ^ ((uint64_t)gg << 16) ^ (uint64_t)i ^ (seed * 0x9E3779B97F4A7C15ULL));
    reinterpret_cast<uint64_t*>(slabs)[w] = mix64(key + (wi + 1) * 0xD1B54A32D192ED03ULL);
  }
}

hipError_t launch_fill_slabs(uint8_t* slabs, uint32_t nslab, uint32_t G, uint32_t E, uint32_t P, uint64_t seed,
                             hipStream_t s) {
  if (!P) return hipSuccess;
  hipLaunchKernelGGL(fill_slabs_kernel, dim3(4096), dim3(256), 0, s, slabs, nslab, G, E, P, seed);
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

// Σ_g max_s committed, on the state a next tick would read (s64_in)
__global__ void sum_committed_kernel(TickParams p, unsigned long long* out) {
  uint64_t acc = 0;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < p.G; g += gridDim.x * blockDim.x) {
    uint64_t m = 0;
    for (uint32_t s = 0; s < p.R; ++s) m = umax64(m, p.s64_in[(uint64_t)S_COMMITTED * p.nrep + (uint64_t)s * p.G + g]);
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
