// raftgpu_apply.hip — committed-entry copy-back: the device side of raftd's apply path.
//
// After each step dragonboat hands a replica's newly committed entries to the state machine
// (rsm → IOnDiskStateMachine.Update), which raftd forwards as POST /UpdateEntries
// (/root/reference/raft/state_machine.go:136-166). Here a tick leaves, per replica, the window
// (apply_lo - 1, applied] it applied (control_kernel; ranges restored from a snapshot excluded:
// those reach the application through RecoverFromSnapshot, not Update). These kernels gather the
// non-empty application entries of that window — config changes and leader no-ops are not
// Update()d — into one contiguous batch so that only newly committed data crosses PCIe, in a
// single hipMemcpyAsync per array.
//
// count_kernel   thread per replica: entries to hand over (coalesced term-ring reads, [L][nrep])
// gather_kernel  wave per replica: ballot-compacted records + 16-B-per-lane payload copies
#include "../../include/raftgpu.h"
#include "raftgpu_internal.h"

namespace rg {

__device__ __forceinline__ bool applies(uint64_t w) { return !(w & TYPE_BIT) && (w & PAY_BIT); }

__global__ void apply_count_kernel(ApplyParams a) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= a.nrep) return;
  const uint32_t s = q / a.G;
  uint32_t c = 0;
  if ((a.slot_mask >> s) & 1u) {
    const uint64_t hi = a.s64[(uint64_t)S_APPLIED * a.nrep + q];
    for (uint64_t i = a.apply_lo[q] > 0 ? a.apply_lo[q] : 1; i <= hi; ++i)
      c += applies(a.tr[(i & (a.L - 1)) * a.nrep + q]) ? 1u : 0u;
  }
  a.cnt[q] = c;
}

__global__ void apply_total_kernel(const uint64_t* off, uint32_t n, uint64_t* total) { *total = off[n]; }

hipError_t launch_apply_count(const ApplyParams& a, uint64_t* total, hipStream_t st) {
  hipLaunchKernelGGL(apply_count_kernel, dim3((a.nrep + 255) / 256), dim3(256), 0, st, a);
  hipError_t r = launch_scan_u32(a.cnt, a.nrep, a.bsum, a.off, st);
  if (r != hipSuccess) return r;
  hipLaunchKernelGGL(apply_total_kernel, dim3(1), dim3(1), 0, st, a.off, a.nrep, total);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256) apply_gather_kernel(ApplyParams a) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint32_t lane = __lane_id();
  const uint32_t q = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  if (q >= a.nrep || a.cnt[q] == 0) return;
  const uint32_t s = q / a.G, j = q - s * a.G;
  const uint64_t n64 = a.nrep, L = a.L, P = a.P, nch = P / 16;
  const uint64_t group = pl_group(a.pl, s, j);
  const uint64_t hi = a.s64[(uint64_t)S_APPLIED * n64 + q];
  uint64_t pos = a.off[q];
  for (uint64_t i0 = a.apply_lo[q] > 0 ? a.apply_lo[q] : 1; i0 <= hi; i0 += 64) {
    const uint64_t i = i0 + lane;
    const uint64_t slot = i & (L - 1);
    const uint64_t w = i <= hi ? a.tr[slot * n64 + q] : 0;
    const bool sel = i <= hi && applies(w);
    const uint64_t mask = __ballot(sel);
    if (sel) {
      const uint64_t k = pos + __builtin_popcountll(mask & ((1ull << lane) - 1));
      const uint2 inf = a.info[((w >> 63) * n64 + q) * L + slot];
      rg_apply_entry r;
      r.index = i;
      r.group = group;
      r.replica_id = s + 1;
      r.len = inf.y & 0xFFFFFF;
      r.crc = inf.x;
      r.rid = j * a.R + s;
      reinterpret_cast<rg_apply_entry*>(a.out_rec)[k] = r;
    }
    // payloads: 16 B per lane over (candidate entry, chunk); unselected candidates idle
    const uint64_t ncand = hi - i0 + 1 < 64 ? hi - i0 + 1 : 64;
    for (uint64_t t = lane; t < ncand * nch; t += 64) {
      const uint64_t e = t / nch, ch = t - e * nch;
      if (!((mask >> e) & 1ull)) continue;
      const uint64_t ie = i0 + e, se = ie & (L - 1);
      const uint64_t we = a.tr[se * n64 + q];
      const uint64_t k = pos + __builtin_popcountll(mask & ((1ull << e) - 1));
      const u32x4 v = *reinterpret_cast<const u32x4*>(a.pay + (((we >> 63) * n64 + q) * L + se) * P + 16 * ch);
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(a.out_pay + k * P + 16 * ch));
    }
    pos += __builtin_popcountll(mask);
  }
}

hipError_t launch_apply_gather(const ApplyParams& a, hipStream_t st) {
  hipLaunchKernelGGL(apply_gather_kernel, dim3((a.nrep + 3) / 4), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace rg
