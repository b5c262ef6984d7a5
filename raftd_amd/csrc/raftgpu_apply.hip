// raftgpu_apply.hip — committed-entry copy-back: the device side of raftd's apply path.
//
// After each step dragonboat hands a replica's newly committed entries to the state machine
// (rsm → IOnDiskStateMachine.Update), which raftd forwards as POST /UpdateEntries
// (/root/reference/raft/state_machine.go:136-166). Here a tick leaves, per replica, the window
// [apply_lo, processed] it handed over, as a length in its hand-off word (feed_word; control_kernel;
// ranges restored from a snapshot excluded:
// those reach the application through RecoverFromSnapshot, not Update). These kernels gather the
// non-empty application entries of that window — config changes and leader no-ops are not
// Update()d — into one contiguous batch so that only newly committed data crosses PCIe, in a
// single hipMemcpyAsync per array.
//
// The batch is ranges, not records: one rg_apply_run per run of consecutive indices (group, replica,
// first index, where its {len, crc} and Cmds start) and 8 B per entry (len, crc) — the index, shard and
// replica of every entry are implied (r05; r04 shipped a 40-B rg_apply_entry per entry).
//
// count_kernel   thread per replica: entries, Cmd chunks and runs to hand over (coalesced [L][nrep] reads)
// gather_kernel  wave per replica: ballot-compacted {len, crc} + run heads, 16-B-per-lane payload copies
// runs_kernel    thread per run: its count (the next run of the replica, or the replica's end, minus it)
#include "../../include/raftgpu.h"
#include "raftgpu_internal.h"

namespace rg {

__device__ __forceinline__ bool applies(uint64_t w) { return !(w & TYPE_BIT) && (w & PAY_BIT); }

__device__ __forceinline__ uint32_t lane_inc_scan(uint32_t v) {
  const uint32_t lane = __lane_id();
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)v, o, 64);
    if (lane >= o) v += y;
  }
  return v;
}

// The Cmds of up to 64 consecutive candidate entries of replica q, packed back to back: lane i holds
// candidate i's inclusive chunk prefix inc (0 chunks if not selected) and its stream position sp;
// chunk t of the run (t < total) belongs to the first candidate whose inc exceeds t (binary search
// over lanes), and is copied from its stream into out + (base + t) · 16.
__device__ __forceinline__ void copy_run(const uint8_t* pool, const uint32_t* pt, uint32_t PTS, uint32_t q,
                                         uint32_t inc, uint32_t sp, uint32_t total, uint8_t* out, uint64_t base) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint32_t lane = __lane_id();
  for (uint32_t t = lane; t < ((total + 63) & ~63u); t += 64) {
    uint32_t lo = 0;  // first lane with inc > t
#pragma unroll
    for (uint32_t step = 32; step; step >>= 1) {
      const uint32_t v = (uint32_t)__shfl((int)inc, (int)(lo + step - 1), 64);
      if (v <= t) lo += step;
    }
    // every lane takes part in the permute: a lane masked off by a branch supplies no data, and a
    // reader of it (lane lo - 1 with its own lo = 0) would get 0
    const uint32_t exl = (uint32_t)__shfl((int)inc, (int)(lo ? lo - 1 : 0), 64);
    const uint32_t ex = lo ? exl : 0u;
    const uint32_t spl = (uint32_t)__shfl((int)sp, (int)(lo < 64 ? lo : 63), 64);
    if (t < total) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(pool + stream_byte(pt, PTS, q, spl + (t - ex)));
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(out + (base + t) * 16));
    }
  }
}

__global__ void apply_count_kernel(ApplyParams a) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= a.nrep) return;
  const uint32_t s = q / a.G;
  uint32_t c = 0, cc = 0, rc = 0;
  if ((a.slot_mask >> s) & 1u) {
    const uint64_t hi = a.s64[(uint64_t)S_PROCESSED * a.nrep + q];
    bool prev = false;
    for (uint64_t i = feed_apply_lo(a.feed[q], hi); i <= hi; ++i) {
      const uint64_t w = a.tr[(i & (a.L - 1)) * a.nrep + q];
      const bool sel = applies(w);
      if (sel) {
        c += 1;
        cc += word_nc(w);
        rc += prev ? 0u : 1u;
      }
      prev = sel;
    }
  }
  a.cnt[q] = c;
  a.ccnt[q] = cc;
  a.rcnt[q] = rc;
}

__global__ void apply_total_kernel(const uint64_t* off, uint32_t n, uint64_t* total) { *total = off[n]; }
__global__ void totals3_kernel(const uint64_t* a, const uint64_t* b, const uint64_t* c, uint32_t n, uint64_t* out) {
  out[0] = a[n];
  out[1] = b[n];
  out[2] = c[n];
}

hipError_t launch_apply_count(const ApplyParams& a, uint64_t* totals, hipStream_t st) {
  hipLaunchKernelGGL(apply_count_kernel, dim3((a.nrep + 255) / 256), dim3(256), 0, st, a);
  hipError_t r = launch_scan_u32(a.cnt, a.nrep, a.bsum, a.off, st);
  if (r == hipSuccess) r = launch_scan_u32(a.ccnt, a.nrep, a.bsum, a.coff, st);
  if (r == hipSuccess) r = launch_scan_u32(a.rcnt, a.nrep, a.bsum, a.roff, st);
  if (r != hipSuccess) return r;
  hipLaunchKernelGGL(totals3_kernel, dim3(1), dim3(1), 0, st, a.off, a.coff, a.roff, a.nrep, totals);
  return hipGetLastError();
}

// wave per replica: ballot-compacted {len, crc}, a run head where a selected entry follows an
// unselected one (or opens the window), then the Cmds of each stretch of 64 candidates packed
__global__ void __launch_bounds__(256) apply_gather_kernel(ApplyParams a) {
  const uint32_t lane = __lane_id();
  const uint32_t q = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  if (q >= a.nrep || a.cnt[q] == 0) return;
  const uint32_t s = q / a.G, j = q - s * a.G;
  const uint64_t n64 = a.nrep, L = a.L;
  const uint64_t group = pl_group(a.pl, s, j);
  const uint64_t hi = a.s64[(uint64_t)S_PROCESSED * n64 + q];
  uint64_t pos = a.off[q], cpos = a.coff[q], rpos = a.roff[q];
  uint64_t carry = 0;  // 1: the candidate before this stretch was selected (its run continues)
  for (uint64_t i0 = feed_apply_lo(a.feed[q], hi); i0 <= hi; i0 += 64) {
    const uint64_t i = i0 + lane;
    const uint64_t slot = i & (L - 1);
    const uint64_t w = i <= hi ? a.tr[slot * n64 + q] : 0;
    const bool sel = i <= hi && applies(w);
    const uint64_t mask = __ballot(sel);
    const uint64_t heads = mask & ~((mask << 1) | carry);
    const uint2 inf = sel ? a.info[((w >> 63) * n64 + q) * L + slot] : make_uint2(0u, 0u);
    const uint32_t nc = sel ? word_nc(w) : 0u, inc = lane_inc_scan(nc);
    const uint64_t below = (1ull << lane) - 1;
    if (sel) {
      const uint64_t k = pos + __builtin_popcountll(mask & below);
      rg_apply_cmd c;
      c.len = word_len(w);
      c.crc = crc_of_cmd(inf.x, c.len, a.P, a.zi);  // the info word keeps the slot CRC
      reinterpret_cast<rg_apply_cmd*>(a.out_cmd)[k] = c;
      if ((heads >> lane) & 1ull) {
        rg_apply_run r;
        r.group = group;
        r.replica_id = s + 1;
        r.rid = j * a.R + s;
        r.first = i;
        r.entry = k;
        r.off = (cpos + inc - nc) * 16;
        r.count = 0;  // runs_kernel
        r._pad = q;   // the replica, for runs_kernel (cleared there)
        reinterpret_cast<rg_apply_run*>(a.out_run)[rpos + __builtin_popcountll(heads & below)] = r;
      }
    }
    const uint32_t total = (uint32_t)__shfl((int)inc, 63, 64);
    if (a.out_pay) copy_run(a.pool, a.pt, a.PTS, q, inc, inf.y, total, a.out_pay, cpos);
    pos += __builtin_popcountll(mask);
    rpos += __builtin_popcountll(heads);
    cpos += total;
    carry = mask >> 63;
  }
}

// a run's entry count: up to the next run of the same replica, else to the replica's last entry
__global__ void apply_runs_kernel(ApplyParams a, uint64_t nruns) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nruns) return;
  rg_apply_run* runs = reinterpret_cast<rg_apply_run*>(a.out_run);
  const uint32_t q = runs[r]._pad;
  const uint64_t end = r + 1 < nruns && runs[r + 1]._pad == q ? runs[r + 1].entry : a.off[q + 1];
  runs[r].count = (uint32_t)(end - runs[r].entry);
}

__global__ void apply_runs_clear_kernel(ApplyParams a, uint64_t nruns) {  // the scratch replica field
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < nruns) reinterpret_cast<rg_apply_run*>(a.out_run)[r]._pad = 0;
}

hipError_t launch_apply_gather(const ApplyParams& a, uint64_t nruns, hipStream_t st) {
  hipLaunchKernelGGL(apply_gather_kernel, dim3((a.nrep + 3) / 4), dim3(256), 0, st, a);
  if (nruns) {
    const dim3 grid((uint32_t)((nruns + 255) / 256));
    hipLaunchKernelGGL(apply_runs_kernel, grid, dim3(256), 0, st, a, nruns);
    hipLaunchKernelGGL(apply_runs_clear_kernel, grid, dim3(256), 0, st, a, nruns);
  }
  return hipGetLastError();
}

// ================================================================== persistence (host WAL feed)
// dragonboat persists Update.EntriesToSave + State{Term, Vote, Commit} (and a snapshot's index)
// before a step's messages leave. Per replica whose log or hard state changed in the last tick:
// one state record, and the entries it rewrote, [persist_lo, last] (full: the whole window), their
// Cmds packed (rg_persist_entry.off).

__device__ __forceinline__ uint64_t persist_first(const PersistParams& a, uint32_t q) {
  const uint64_t n = a.nrep, marker = a.s64[(uint64_t)S_MARKER * n + q];
  const uint64_t lo = a.full ? marker + 1 : feed_persist_lo(a.feed[q], a.s64[(uint64_t)S_LAST * n + q]);
  return lo > marker ? lo : marker + 1;
}

__global__ void persist_count_kernel(PersistParams a) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= a.nrep) return;
  if (!((a.slot_mask >> (q / a.G)) & 1u)) {  // another node's replica: not this hand-off's to persist
    a.scnt[q] = a.ecnt[q] = a.ccnt[q] = a.tcnt[q] = 0;
    return;
  }
  const uint64_t n = a.nrep;
  const uint64_t last = a.s64[(uint64_t)S_LAST * n + q], lo = persist_first(a, q);
  const uint32_t ne = lo <= last ? (uint32_t)(last - lo + 1) : 0u;
  // the step recorded whether it wrote entries or changed the hard state (no previous state to diff)
  const bool changed = a.full || ne > 0 || (a.feed[q] & FEED_PERSIST);
  uint32_t cc = 0, tc = 0;
  uint64_t pt = ~0ull;
  for (uint64_t i = lo; i <= last; ++i) {
    const uint64_t w = a.tr[(i & (a.L - 1)) * n + q];
    cc += word_nc(w);
    tc += (w & TERM_MASK) != pt ? 1u : 0u;  // a term run starts
    pt = w & TERM_MASK;
  }
  a.scnt[q] = changed ? 1u : 0u;
  a.ecnt[q] = ne;
  a.ccnt[q] = cc;
  a.tcnt[q] = tc;
}

__global__ void persist_total_kernel(const PersistParams a, uint64_t* totals) {
  totals[0] = a.soff[a.nrep];
  totals[1] = a.eoff[a.nrep];
  totals[2] = a.coff[a.nrep];
  totals[3] = a.toff[a.nrep];
}

hipError_t launch_persist_count(const PersistParams& a, uint64_t* totals, hipStream_t st) {
  hipLaunchKernelGGL(persist_count_kernel, dim3((a.nrep + 255) / 256), dim3(256), 0, st, a);
  hipError_t r = launch_scan_u32(a.scnt, a.nrep, a.bsum, a.soff, st);
  if (r == hipSuccess) r = launch_scan_u32(a.ecnt, a.nrep, a.bsum, a.eoff, st);
  if (r == hipSuccess) r = launch_scan_u32(a.ccnt, a.nrep, a.bsum, a.coff, st);
  if (r == hipSuccess) r = launch_scan_u32(a.tcnt, a.nrep, a.bsum, a.toff, st);
  if (r != hipSuccess) return r;
  hipLaunchKernelGGL(persist_total_kernel, dim3(1), dim3(1), 0, st, a, totals);
  return hipGetLastError();
}

__global__ void persist_state_kernel(PersistParams a) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= a.nrep || !a.scnt[q]) return;
  const uint64_t n = a.nrep;
  const uint32_t s = q / a.G, j = q - s * a.G;
  const uint64_t* v = a.s64 + q;
  rg_persist_state r;
  r.group = pl_group(a.pl, s, j);
  r.replica_id = s + 1;
  r.rid = j * a.R + s;
  r.term = v[S_TERM * n];
  r.vote = v[S_VOTE * n];
  r.commit = v[S_COMMITTED * n];
  r.last = v[S_LAST * n];
  r.marker = v[S_MARKER * n];
  r.marker_term = v[S_MARKER_TERM * n];
  r.snap_index = v[S_SNAP_INDEX * n];
  r.snap_term = v[S_SNAP_TERM * n];
  r.first = persist_first(a, q);
  r.entry_off = a.eoff[q];
  r.members = a.s32[(uint64_t)S_MEMBERS * n + q];
  r.snap_members = a.s32[(uint64_t)S_SNAP_MEMBERS * n + q];
  r.payload_off = a.coff[q] * 16;
  r.term_off = a.toff[q];
  r.n_terms = a.tcnt[q];
  r._pad = 0;
  reinterpret_cast<rg_persist_state*>(a.out_state)[a.soff[q]] = r;
}

__global__ void __launch_bounds__(256) persist_entries_kernel(PersistParams a) {
  const uint32_t lane = __lane_id();
  const uint32_t q = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  if (q >= a.nrep || a.ecnt[q] == 0) return;
  const uint32_t s = q / a.G, j = q - s * a.G;
  const uint64_t n64 = a.nrep, L = a.L;
  const uint64_t lo = persist_first(a, q), hi = a.s64[(uint64_t)S_LAST * n64 + q];
  const uint64_t base = a.eoff[q];
  uint64_t cpos = a.coff[q], tpos = a.toff[q];
  uint64_t prev = ~0ull;  // the term of the entry before this stretch (~0: none yet)
  rg_persist_term* terms = reinterpret_cast<rg_persist_term*>(a.out_term);
  (void)s; (void)j;
  for (uint64_t i0 = lo; i0 <= hi; i0 += 64) {
    const uint64_t i = i0 + lane;
    const bool in = i <= hi;
    const uint32_t nin = (uint32_t)(hi - i0 + 1 < 64 ? hi - i0 + 1 : 64);
    const uint64_t slot = i & (L - 1), w = in ? a.tr[slot * n64 + q] : 0;
    const uint2 inf = in ? a.info[((w >> 63) * n64 + q) * L + slot] : make_uint2(0u, 0u);
    const uint32_t nc = word_nc(w), inc = lane_inc_scan(nc);
    const uint64_t tm = w & TERM_MASK;
    // term runs: a head where the term differs from the previous entry's (lane 0: the last stretch's)
    const uint32_t up = (uint32_t)__shfl_up((int)(uint32_t)tm, 1, 64), uph = (uint32_t)__shfl_up((int)(uint32_t)(tm >> 32), 1, 64);
    const uint64_t before = lane ? ((uint64_t)uph << 32 | up) : prev;
    const uint64_t heads = __ballot(in && tm != before);
    if (in) {
      rg_persist_entry r;
      r.len = (w & TYPE_BIT) ? (RG_PERSIST_CONFIG | word_len(w)) : (w & PAY_BIT) ? word_len(w) : 0u;
      r.crc = (w & PAY_BIT) ? crc_of_cmd(inf.x, word_len(w), a.P, a.zi) : 0u;
      reinterpret_cast<rg_persist_entry*>(a.out_ent)[base + (i - lo)] = r;
      if ((heads >> lane) & 1ull) {  // count: its first entry's position for now (persist_terms_kernel)
        rg_persist_term t;
        t.term = tm;
        t.count = base + (i - lo);
        terms[tpos + __builtin_popcountll(heads & ((1ull << lane) - 1))] = t;
      }
    }
    const uint32_t total = (uint32_t)__shfl((int)inc, 63, 64);
    copy_run(a.pool, a.pt, a.PTS, q, inc, inf.y, total, a.out_pay, cpos);
    cpos += total;
    tpos += __builtin_popcountll(heads);
    const uint32_t ll = (uint32_t)__shfl((int)(uint32_t)tm, (int)(nin - 1), 64), lh = (uint32_t)__shfl((int)(uint32_t)(tm >> 32), (int)(nin - 1), 64);
    prev = (uint64_t)lh << 32 | ll;
  }
}

// thread per replica: its term runs' counts from their first entries' positions
__global__ void persist_terms_kernel(PersistParams a) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= a.nrep || !a.tcnt[q]) return;
  rg_persist_term* t = reinterpret_cast<rg_persist_term*>(a.out_term) + a.toff[q];
  const uint32_t n = a.tcnt[q];
  for (uint32_t k = 0; k < n; ++k) {
    const uint64_t end = k + 1 < n ? t[k + 1].count : a.eoff[q] + a.ecnt[q];
    t[k].count = end - t[k].count;
  }
}

hipError_t launch_persist_gather(const PersistParams& a, hipStream_t st) {
  hipLaunchKernelGGL(persist_state_kernel, dim3((a.nrep + 255) / 256), dim3(256), 0, st, a);
  hipLaunchKernelGGL(persist_entries_kernel, dim3((a.nrep + 3) / 4), dim3(256), 0, st, a);
  hipLaunchKernelGGL(persist_terms_kernel, dim3((a.nrep + 255) / 256), dim3(256), 0, st, a);
  return hipGetLastError();
}

// ================================================================== snapshot events
// the step leaves FEED_RESTORED / FEED_TAKEN in feed[q] per replica; compact the
// non-zero ones (thread per replica, coalesced) into rg_snapshot_event records.

__global__ void snap_count_kernel(SnapParams a) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= a.nrep) return;
  a.cnt[q] = ((a.slot_mask >> (q / a.G)) & 1u) && (a.feed[q] & (FEED_RESTORED | FEED_TAKEN)) ? 1u : 0u;
}

hipError_t launch_snap_count(const SnapParams& a, uint64_t* total, hipStream_t st) {
  hipLaunchKernelGGL(snap_count_kernel, dim3((a.nrep + 255) / 256), dim3(256), 0, st, a);
  hipError_t r = launch_scan_u32(a.cnt, a.nrep, a.bsum, a.off, st);
  if (r != hipSuccess) return r;
  hipLaunchKernelGGL(apply_total_kernel, dim3(1), dim3(1), 0, st, a.off, a.nrep, total);
  return hipGetLastError();
}

__global__ void snap_gather_kernel(SnapParams a) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= a.nrep || !a.cnt[q]) return;
  const uint64_t n = a.nrep, ev = a.feed[q];
  const uint64_t restored = feed_restored_at(ev, a.s64[(uint64_t)S_PROCESSED * n + q]);
  const uint32_t s = q / a.G, j = q - s * a.G;
  rg_snapshot_event r;
  r.group = pl_group(a.pl, s, j);
  r.replica_id = s + 1;
  r.rid = j * a.R + s;
  r.kind = (ev & FEED_RESTORED ? RG_SNAP_RESTORED : 0u) | ((ev & FEED_TAKEN) ? RG_SNAP_TAKEN : 0u);
  r._pad = 0;
  r.restored = restored;
  r.index = (ev & FEED_TAKEN) ? a.s64[(uint64_t)S_SNAP_INDEX * n + q] : 0;
  r.term = (ev & FEED_TAKEN) ? a.s64[(uint64_t)S_SNAP_TERM * n + q] : 0;
  reinterpret_cast<rg_snapshot_event*>(a.out)[a.off[q]] = r;
}

hipError_t launch_snap_gather(const SnapParams& a, hipStream_t st) {
  hipLaunchKernelGGL(snap_gather_kernel, dim3((a.nrep + 255) / 256), dim3(256), 0, st, a);
  return hipGetLastError();
}

// ================================================================== ReadIndex results
// reads made ready in the last tick: RD_TICK == the number of ticks run (read_ready stores tick + 1)
__global__ void read_count_kernel(SnapParams a) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= a.nrep) return;
  a.cnt[q] = ((a.slot_mask >> (q / a.G)) & 1u) && a.rdst[(uint64_t)RD_TICK * a.nrep + q] == a.tick
                ? (uint32_t)min(a.rdst[(uint64_t)RD_N * a.nrep + q], (uint64_t)RG_RQ)
                : 0u;
}

hipError_t launch_read_count(const SnapParams& a, uint64_t* total, hipStream_t st) {
  hipLaunchKernelGGL(read_count_kernel, dim3((a.nrep + 255) / 256), dim3(256), 0, st, a);
  hipError_t r = launch_scan_u32(a.cnt, a.nrep, a.bsum, a.off, st);
  if (r != hipSuccess) return r;
  hipLaunchKernelGGL(apply_total_kernel, dim3(1), dim3(1), 0, st, a.off, a.nrep, total);
  return hipGetLastError();
}

__global__ void read_gather_kernel(SnapParams a) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= a.nrep || !a.cnt[q]) return;
  const uint32_t s = q / a.G, j = q - s * a.G;
  rg_read_ready r;
  r.group = pl_group(a.pl, s, j);
  r.replica_id = s + 1;
  r.rid = j * a.R + s;
  for (uint32_t k = 0; k < a.cnt[q]; ++k) {  // in the order they became ready
    r.ctx = a.rdst[(uint64_t)(RD_CTX + k) * a.nrep + q];
    r.index = a.rdst[(uint64_t)(RD_INDEX + k) * a.nrep + q];
    reinterpret_cast<rg_read_ready*>(a.out)[a.off[q] + k] = r;
  }
}

hipError_t launch_read_gather(const SnapParams& a, hipStream_t st) {
  hipLaunchKernelGGL(read_gather_kernel, dim3((a.nrep + 255) / 256), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace rg
