// raftgpu_ctl.hip — control_kernel<R> (all Raft logic, one lane per replica) and the
// resident multi-tick control kernel, one instantiation per translation unit: the build compiles this
// file once per replica count (-DRG_CTL_R=1..8), so the eight register-heavy instantiations compile in
// parallel. The step itself is raftgpu_control.h (shared with the CPU harness tests/native/ctl_host.cpp).
#include "raftgpu_control.h"
#include "raftgpu_dev.h"

#ifndef RG_CTL_R
#error "compile raftgpu_ctl.hip with -DRG_CTL_R=<replicas> (raftd_amd/build.py)"
#endif

namespace rg {

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
// The checksum: lane i loads word i (one coalesced 424-B wave load, through a laundered pointer so
// it stays separate from the step's scalar field reads) and the wave sums the terms with a
// butterfly. r03a's volatile chain cost 53 dependent cache-bypassing loads per wave; a chain of
// seven s_load_dwordx16 (r03b) still waited seven scalar round trips at the head of every wave.
// On a mismatch the first lane of the launch reports it (sticky *perr) and every wave returns.
__device__ __forceinline__ bool tp_verify(const TickParams* pp, uint32_t* perr, uint32_t q, const char* kname) {
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
      printf("raftgpu: %s parameter block checksum mismatch (tick %llu): launch skipped\n", kname,
             (unsigned long long)pp->tick);
      atomicOr(perr, 1u);
    }
    return false;
  }
  return true;
}

template <int R>
__global__ void __launch_bounds__(RG_CTL_BLOCK, RG_CTL_MINWAVES) control_kernel(const TickParams* __restrict__ pp,
                                                                               uint32_t* perr) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (!tp_verify(pp, perr, q, "control_kernel")) return;
  CTickParams& cp = *(CTickParams*)pp;
  if (q >= cp.nrep) return;
#ifdef RG_CTL_PROFILE
  const uint32_t t0 = (uint32_t)__builtin_amdgcn_s_memtime();
  Ctl<R, false, -1, false, true> c(cp, q);
  c.stamps[0] = t0;
#else
  Ctl<R, false, -1, false, true> c(cp, q);
#endif
  c.run();
}

// ---- the fast path (DESIGN.md §3 "Fast path"): Ctl<R, true> steps every replica through the
// steady-state branches only and hands a replica whose step leaves them to the slow kernel, which
// re-runs that replica's whole step with the full Ctl<R> (an aborted fast step stored nothing).
#ifndef RG_CTL_FAST_WAVES
#define RG_CTL_FAST_WAVES (RG_CTL_R <= 4 ? 3 : 2)  // the most waves per SIMD without scratch (r06: 145 VGPRs at R 3, 221 at R 8)
#endif
// The fast path is compiled once per role — Ctl<R, true, LEADER> for leaders, Ctl<R, true, FOLLOWER>
// for every other replica (followers step, candidates hand off) — and each lane runs its role's
// step: the two are separate branches, so the kernel holds the larger role's live values instead of
// both roles' at once (r04: 204 -> 168 VGPRs at R = 3, three waves per SIMD). In steady state a wave's
// lanes share a role (slot-major lanes, one leader slot per group) and run one branch.
// one replica's fast step (its role's instantiation); returns whether it left the fast path. LAT: the
// latency build of small engines (every field loaded up front, Ctl's LAT)
template <int R, bool LAT = false>
__device__ __forceinline__ bool fast_step(CTickParams& cp, uint32_t q) {
  if (cp.s32[(uint64_t)S_ROLE * cp.nrep + q] == LEADER) {
#ifdef RG_CTL_PROFILE
    const uint32_t t0 = (uint32_t)__builtin_amdgcn_s_memtime();
    Ctl<R, true, LEADER, LAT> c(cp, q);
    c.stamps[0] = t0;
#else
    Ctl<R, true, LEADER, LAT> c(cp, q);
#endif
    c.run();
    return c.aborted;
  }
#ifdef RG_CTL_PROFILE
  const uint32_t t0 = (uint32_t)__builtin_amdgcn_s_memtime();
  Ctl<R, true, FOLLOWER, LAT> c(cp, q);
  c.stamps[0] = t0;
#else
  Ctl<R, true, FOLLOWER, LAT> c(cp, q);
#endif
  c.run();
  return c.aborted;
}

// the hand-off count (measurement: rg_debug_ctl_slow): one atomic per wave with aborted lanes
__device__ __forceinline__ uint32_t count_slow(CTickParams& cp, bool aborted) {
  const uint64_t m = __ballot(aborted);
  uint32_t base = 0;
  if (m) {
    const uint32_t first = (uint32_t)__ffsll((long long)m) - 1;
    if ((threadIdx.x & 63u) == first) base = atomicAdd(cp.slow_cnt + (cp.tick & 1), (uint32_t)__popcll(m));
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)first);
  }
  return base;
}
// the hand-off list: an aborted lane's replica at base + its rank among the wave's aborted lanes
__device__ __forceinline__ void list_slow(CTickParams& cp, bool aborted, uint32_t base, uint32_t q) {
  const uint64_t m = __ballot(aborted);
  if (aborted) cp.slow_flag[base + (uint32_t)__popcll(m & ((1ull << (threadIdx.x & 63u)) - 1))] = q;
}

// RG_AB_CTL2D (diagnostic variant, never the product): the fast and slow kernels on r04f's (column,
// slot) grid, the slot index blockIdx.y — the launch geometry of the r04 memory-aperture fault
// ("The control-kernel fault"). q is still slot · G + column.
#ifdef RG_AB_CTL2D
#define RG_CTL_Q (blockIdx.y * ((const TickParams*)pp)->G + blockIdx.x * blockDim.x + threadIdx.x)
#define RG_CTL_COL_OK(cp) (blockIdx.x * blockDim.x + threadIdx.x < (cp).G)
#else
#define RG_CTL_Q (blockIdx.x * blockDim.x + threadIdx.x)
#define RG_CTL_COL_OK(cp) true
#endif
#ifndef RG_SLOW_GRID
#define RG_SLOW_GRID 1024u  // workgroups of control_slow_kernel (at most): 256 CUs x 4 SIMDs
#endif
template <int R>
__global__ void __launch_bounds__(RG_CTL_BLOCK, RG_CTL_FAST_WAVES) control_fast_kernel(
    const TickParams* __restrict__ pp, uint32_t* perr) {
  const uint32_t q = RG_CTL_Q;
  if (!tp_verify(pp, perr, q, "control_fast_kernel")) return;
  CTickParams& cp = *(CTickParams*)pp;
  if (q == 0) cp.slow_cnt[(cp.tick + 1) & 1] = 0;  // the next tick's counter (its last reader ran before us)
  if (q >= cp.nrep || !RG_CTL_COL_OK(cp)) return;
  const bool aborted = fast_step<R>(cp, q);
#ifdef RG_AB_CTL2D
  cp.slow_flag[q] = aborted ? 1u : 0u;  // for control_slow_kernel (the diagnostic 2-D grid)
  count_slow(cp, aborted);
#else
  list_slow(cp, aborted, count_slow(cp, aborted), q);
#endif
}

// Small engines (a wave or less per SIMD: occupancy buys nothing) run the fallback in the same
// launch: a lane that leaves the fast path re-runs its step with the full Ctl<R> right away, and the
// tick saves the slow kernel's launch (C2 shapes: the tick is a few of these latencies).
#if RG_CTL_R <= 5
template <int R>
__global__ void __launch_bounds__(RG_CTL_BLOCK, 1) control_fastfb_kernel(const TickParams* __restrict__ pp,
                                                                         uint32_t* perr) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (!tp_verify(pp, perr, q, "control_fastfb_kernel")) return;
  CTickParams& cp = *(CTickParams*)pp;
  if (q == 0) cp.slow_cnt[(cp.tick + 1) & 1] = 0;
  if (q >= cp.nrep) return;
  const bool aborted = fast_step<R, true>(cp, q);
  count_slow(cp, aborted);
  if (aborted) {  // the fast step stored nothing: the full step from the same inputs
    Ctl<R> c(cp, q);
    c.run();
  }
}
#endif

// the replicas the fast kernel handed off this tick (a wave without one leaves at once). Lane q steps
// replica q, as control_kernel does (a one-dimensional grid: the full step with a grid-uniform slot
// index, blockIdx.y, faulted in the full-size C3 test in r04; this mapping has run every suite since r01).
template <int R>
__global__ void __launch_bounds__(RG_CTL_BLOCK, RG_CTL_MINWAVES) control_slow_kernel(const TickParams* __restrict__ pp,
                                                                                    uint32_t* perr) {
#ifdef RG_AB_CTL2D
  const uint32_t q = RG_CTL_Q;
  if (!tp_verify(pp, perr, q, "control_slow_kernel")) return;
  CTickParams& cp = *(CTickParams*)pp;
  if (q >= cp.nrep || !RG_CTL_COL_OK(cp) || !cp.slow_flag[q]) return;
#if !defined(RG_AB_CTL2D_Q)
  Ctl<R, false, -1, false, true> c(cp, blockIdx.y, blockIdx.x * blockDim.x + threadIdx.x);  // the slot a grid-uniform scalar
#else  // RG_AB_CTL2D_Q: the 2-D launch, the slot derived from q (a per-lane value to the compiler)
  Ctl<R, false, -1, false, true> c(cp, q);
#endif
  c.run();
#else
  // the list the fast kernel wrote: lane i of the grid steps entries i, i + grid, ... (every replica once)
  const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
  if (!tp_verify(pp, perr, i0, "control_slow_kernel")) return;
  CTickParams& cp = *(CTickParams*)pp;
  // the count is re-read after each step (a scalar-cache hit) instead of living through it: with it and
  // the list index both live, the full step spilled four VGPRs at R <= 5 (and to scratch at R = 7)
  auto count = [&]() -> uint32_t {
    RG_G(uint32_t) c = cp.slow_cnt;
    asm volatile("" : "+s"(c));
    return c[cp.tick & 1];
  };
#if RG_CTL_R <= 5
  for (uint32_t i = i0; i < count() && i < cp.nrep; i += gridDim.x * blockDim.x) {
    Ctl<R, false, -1, false, true> c(cp, cp.slow_flag[i]);
    c.run();
  }
#else  // R 6-8: one entry per lane, a full grid (the loop needed scratch at R = 7)
  if (i0 < count() && i0 < cp.nrep) {
    Ctl<R, false, -1, false, true> c(cp, cp.slow_flag[i0]);
    c.run();
  }
#endif
#endif
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
      if (fast_step<R, true>(cp[i], q)) {  // left the fast path (stored nothing): the full step
        Ctl<R> c(cp[i], q);
        c.run();
      }
    }
    __syncthreads();  // tick i's outboxes and state, written by this workgroup, before tick i + 1 reads them
  }
}

template <>
hipError_t launch_control_t<RG_CTL_R>(const TickParams* p, uint32_t* perr, uint32_t nrep, hipStream_t s) {
#ifdef RG_DEV_NO_CONTROL  // development builds of the other kernels only (ISA / resource checks)
  (void)p; (void)perr; (void)nrep; (void)s;
  return hipErrorInvalidValue;
#else
  hipLaunchKernelGGL(control_kernel<RG_CTL_R>, dim3((nrep + RG_CTL_BLOCK - 1) / RG_CTL_BLOCK), dim3(RG_CTL_BLOCK), 0, s,
                     p, perr);
  return hipGetLastError();
#endif
}

template <>
hipError_t launch_control_fast_t<RG_CTL_R>(const TickParams* p, uint32_t* perr, uint32_t nrep, bool fb, hipStream_t s) {
#if defined(RG_DEV_NO_CONTROL) || !defined(RG_CTL_FASTREP)  // the fast path builds on the uniform Replicate
  (void)p; (void)perr; (void)nrep; (void)fb; (void)s;
  return hipErrorInvalidValue;
#else
  const dim3 grid((nrep + RG_CTL_BLOCK - 1) / RG_CTL_BLOCK), block(RG_CTL_BLOCK);
#if RG_CTL_R <= 5  // R 6-8: the fast and the full step together need scratch
  if (fb) {
    hipLaunchKernelGGL(control_fastfb_kernel<RG_CTL_R>, grid, block, 0, s, p, perr);
    return hipGetLastError();
  }
#else
  (void)fb;
#endif
#ifdef RG_AB_CTL2D
  const dim3 g2((nrep / RG_CTL_R + RG_CTL_BLOCK - 1) / RG_CTL_BLOCK, RG_CTL_R);
  hipLaunchKernelGGL(control_fast_kernel<RG_CTL_R>, g2, block, 0, s, p, perr);
  hipLaunchKernelGGL(control_slow_kernel<RG_CTL_R>, g2, block, 0, s, p, perr);
#else
  hipLaunchKernelGGL(control_fast_kernel<RG_CTL_R>, grid, block, 0, s, p, perr);
  // the hand-off list's walk: one full-step wave per SIMD fills the chip (256 VGPRs, occupancy 1)
  const dim3 sgrid(RG_CTL_R > 5 || grid.x < RG_SLOW_GRID ? grid.x : RG_SLOW_GRID);
  hipLaunchKernelGGL(control_slow_kernel<RG_CTL_R>, sgrid, block, 0, s, p, perr);
#endif
  return hipGetLastError();
#endif
}

template <>
hipError_t launch_control_resident_t<RG_CTL_R>(const TickParams* p, uint32_t k, uint32_t* perr, uint32_t G,
                                              hipStream_t s) {
#if defined(RG_DEV_NO_CONTROL) || defined(RG_CTL_NO_RESIDENT) || RG_CTL_R > 4
  // R > 4: a control wave needs a SIMD of its own (occupancy 1), and a CU has four
  (void)p; (void)k; (void)perr; (void)G; (void)s;
  return hipErrorInvalidValue;
#else
  hipLaunchKernelGGL(control_resident_kernel<RG_CTL_R>, dim3((G + 63) / 64), dim3(64 * RG_CTL_R), 0, s, p, k, perr);
  return hipGetLastError();
#endif
}

}  // namespace rg
