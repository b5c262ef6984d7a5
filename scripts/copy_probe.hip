// Streaming-copy shapes on this box (measurement tool behind rg_probe_copy's choice of shape).
// build: hipcc --offload-arch=gfx950 -O3 scripts/copy_probe.hip -o scripts/copy_probe
#include <hip/hip_runtime.h>

#include <cstdio>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// A: grid-stride, U loads per lane spaced a whole grid apart
template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_gs(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  const uint64_t st = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * st < n; i += U * st) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(s + i + u * st) : s[i + u * st];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], d + i + u * st);
      else d[i + u * st] = v[u];
    }
  }
}

// B: block tiles of 256 * U contiguous vectors, grid-stride over tiles
template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_tile(const u32x4* __restrict__ s, u32x4* __restrict__ d, uint64_t n) {
  const uint64_t tile = 256ull * U;
  for (uint64_t b = (uint64_t)blockIdx.x * tile; b + tile <= n; b += (uint64_t)gridDim.x * tile) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = NT ? __builtin_nontemporal_load(s + b + u * 256 + threadIdx.x) : s[b + u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], d + b + u * 256 + threadIdx.x);
      else d[b + u * 256 + threadIdx.x] = v[u];
    }
  }
}

template <class K>
static void run(const char* name, K k, int grid, const u32x4* a, u32x4* b, uint64_t n) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e9;
  for (int r = 0; r < 8; ++r) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, a, b, n);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (r && ms < best) best = ms;
  }
  printf("%-30s grid %8d  %7.1f GB/s\n", name, grid, 2.0 * n * 16 / (best / 1e3) / 1e9);
}

int main() {
  const uint64_t bytes = 4ull << 30, n = bytes / 16;
  u32x4 *a, *b;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
  (void)hipMemset(a, 1, bytes);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int per : {4, 8, 16}) {
    run("grid-stride U4 nt", copy_gs<4, true>, cus * per, a, b, n);
    run("grid-stride U4 plain", copy_gs<4, false>, cus * per, a, b, n);
    run("grid-stride U8 nt", copy_gs<8, true>, cus * per, a, b, n);
    run("tile U4 nt", copy_tile<4, true>, cus * per, a, b, n);
    run("tile U8 nt", copy_tile<8, true>, cus * per, a, b, n);
    run("tile U8 plain", copy_tile<8, false>, cus * per, a, b, n);
    run("tile U16 nt", copy_tile<16, true>, cus * per, a, b, n);
  }
  run("tile U8 nt, one tile/block", copy_tile<8, true>, (int)(n / 2048), a, b, n);
  run("tile U4 plain, one tile/block", copy_tile<4, false>, (int)(n / 1024), a, b, n);
  return 0;
}
