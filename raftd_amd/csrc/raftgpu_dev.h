// raftgpu_dev.h — wave-level helpers shared by the kernel translation units (device code only).
#pragma once
#include "raftgpu_internal.h"

namespace rg {

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ uint32_t wave_excl_scan32(uint32_t v) {
  const uint32_t lane = lane_id();
  uint32_t x = v;
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
    if (lane >= o) x += y;
  }
  return x - v;
}

}  // namespace rg
