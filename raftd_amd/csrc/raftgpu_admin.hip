// raftgpu_admin.hip — small gather / scatter kernels behind rg_read_*, rg_import_replica and
// rg_deliver: they translate between the device's structure-of-arrays layout (slot-major
// replica numbering q = s·G + g) and the C-ABI's per-replica views (rid = g·R + s).
// Not on the tick path.
#include <algorithm>

#include "../../include/raftgpu.h"
#include "raftgpu_internal.h"

namespace rg {

__device__ __forceinline__ uint32_t q_of(const TickParams& t, uint32_t rid) {
  const uint32_t g = rid / t.R, s = rid - g * t.R;
  return s * t.G + g;
}

__global__ void gather_replicas_kernel(AdminParams a, uint32_t first, uint32_t n, rg_replica_view* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const TickParams& t = a.t;
  const uint32_t q = q_of(t, first + i);
  const uint64_t N = t.nrep;
  rg_replica_view v;
  const uint64_t* s64 = t.s64 + q;
  const uint32_t* s32 = t.s32 + q;
  v.term = s64[S_TERM * N]; v.vote = s64[S_VOTE * N]; v.leader = s64[S_LEADER * N];
  v.committed = s64[S_COMMITTED * N]; v.applied = s64[S_APPLIED * N]; v.last = s64[S_LAST * N];
  v.marker = s64[S_MARKER * N]; v.marker_term = s64[S_MARKER_TERM * N]; v.snap_index = s64[S_SNAP_INDEX * N];
  v.snap_term = s64[S_SNAP_TERM * N]; v.cap_base = s64[S_CAP_BASE * N]; v.processed = s64[S_PROCESSED * N];
  v.role = s32[S_ROLE * N]; v.election_tick = s32[S_ETICK * N]; v.heartbeat_tick = s32[S_HTICK * N];
  v.rand_timeout = s32[S_RAND_TO * N]; v.rng_ctr = s32[S_RNG_CTR * N]; v.granted = s32[S_GRANTED * N];
  v.responded = s32[S_RESPONDED * N]; v.active = s32[S_ACTIVE * N];
  v.err = s32[S_ERR * N] | a.crc_err[q];
  v.drops = s32[S_DROPS * N];
  v.members = s32[S_MEMBERS * N]; v.snap_members = s32[S_SNAP_MEMBERS * N]; v.cc_pending = s32[S_CC_PENDING * N];
  v._mpad = 0;
  for (uint32_t j = 0; j < RG_MAX_REPLICAS; ++j) {
    const bool in = j < t.R;
    v.match[j] = in ? t.rem[(0 * t.R + j) * N + q] : 0;
    v.next[j] = in ? t.rem[(1 * t.R + j) * N + q] : 0;
    v.rsnap[j] = in ? t.rem[(2 * t.R + j) * N + q] : 0;
    v.rstate[j] = in ? t.rst[j * N + q] : 0;
  }
  out[i] = v;
}

hipError_t launch_gather_replicas(const AdminParams& a, uint32_t first, uint32_t n, void* out, hipStream_t s) {
  hipLaunchKernelGGL(gather_replicas_kernel, dim3((n + 63) / 64), dim3(64), 0, s, a, first, n,
                     (rg_replica_view*)out);
  return hipGetLastError();
}

// the last tick's messages rid → dst: the outbox as the next tick will read it (hdr_in / mt_in)
__global__ void gather_msgs_kernel(AdminParams a, uint32_t rid, uint32_t dst, uint64_t* out_hdr, uint64_t* out_terms,
                                   uint32_t* out_cnt) {
  const TickParams& t = a.t;
  const uint32_t g = rid / t.R, s = rid - g * t.R;
  const uint64_t plane = (uint64_t)t.R * t.R * t.K * t.G;
  const uint32_t cnt = cnt_n(t.cnt_in[((uint64_t)s * t.R + dst) * t.G + g]);
  const uint32_t k = threadIdx.x;
  if (k == 0) *out_cnt = cnt;
  if (k >= cnt || k >= t.K) return;
  const uint64_t* h = t.hdr_in + (((uint64_t)s * t.R + dst) * t.K + k) * t.G + g;
  const uint64_t* mt = t.mt_in + ((((uint64_t)s * t.R + dst) * t.K + k) * t.E) * t.G + g;
  const uint32_t type = (uint32_t)(h[0] & 0xFF), n = (uint32_t)(h[0] >> 32);
  // a uniform Replicate (RG_UNIFORM in word 7, its Cmds' stream position in word 5) is shown
  // expanded, as the message it encodes
  const bool uni = type == M_REPLICATE && ((uint32_t)h[7 * plane] & RG_UNIFORM);
  // a Propose's word 4 carries its batch's stream layout (raftgpu_control.h), not a commit index
  const bool prop = type == M_PROPOSE;
  const uint32_t wm = hdr_words(type, n);  // the words the message carries; the others read as 0
  for (int w = 0; w < 8; ++w)
    out_hdr[k * 8 + w] = (uni && w == 5) || (prop && w == 4) || !((wm >> w) & 1u)
                             ? 0ull
                             : h[w * plane] & (w == 7 && uni ? ~(uint64_t)RG_UNIFORM : ~0ull);
  for (uint32_t e = 0; e < t.E; ++e)
    out_terms[(uint64_t)k * t.E + e] =
        (type == M_REPLICATE && e < n) ? (mt[uni ? 0 : (uint64_t)e * t.G] & TERM_MASK) : 0;
}

hipError_t launch_gather_msgs(const AdminParams& a, uint32_t rid, uint32_t dst, void* out_hdr, uint64_t* out_terms,
                              uint32_t* out_cnt, hipStream_t s) {
  hipLaunchKernelGGL(gather_msgs_kernel, dim3(1), dim3(64), 0, s, a, rid, dst, (uint64_t*)out_hdr, out_terms,
                     out_cnt);
  return hipGetLastError();
}

// one thread per entry: its view
__global__ void gather_entries_kernel(AdminParams a, uint32_t rid, uint64_t first, uint32_t n, rg_entry_view* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const TickParams& t = a.t;
  const uint32_t q = q_of(t, rid);
  const uint64_t slot = (first + i) & (t.L - 1);
  const uint64_t w = t.tr[slot * t.nrep + q];
  const uint64_t bank = w >> 63;
  const uint2 inf = a.info[(bank * t.nrep + q) * t.L + slot];
  rg_entry_view v;
  v.term = w & TERM_MASK;
  v.type = (uint32_t)((w >> 61) & 1);
  v.len = (w & (PAY_BIT | TYPE_BIT)) ? word_len(w) : 0u;  // a ConfigChange reports its descriptor
  v.crc = (w & PAY_BIT) ? crc_of_cmd(inf.x, v.len, t.P, a.zi) : 0u;  // the info word keeps the slot CRC
  v.bank = (uint32_t)bank;
  out[i] = v;
}

hipError_t launch_gather_entries(const AdminParams& a, uint32_t rid, uint64_t first, uint32_t n, void* out,
                                 hipStream_t s) {
  hipLaunchKernelGGL(gather_entries_kernel, dim3((n + 63) / 64), dim3(64), 0, s, a, rid, first, n,
                     (rg_entry_view*)out);
  return hipGetLastError();
}

// one block per entry: its Cmd's chunks, read through the stream's pages, to out + ao[i] (16-B aligned;
// ao[i] = ~0: no Cmd)
__global__ void __launch_bounds__(256) gather_cmds_kernel(AdminParams a, uint32_t rid, uint64_t first,
                                                          const uint64_t* ao, uint8_t* out) {
  const uint32_t i = blockIdx.x;
  if (ao[i] == ~0ull) return;
  const TickParams& t = a.t;
  const uint32_t q = q_of(t, rid);
  const uint64_t slot = (first + i) & (t.L - 1);
  const uint64_t w = t.tr[slot * t.nrep + q];
  const uint2 inf = a.info[((w >> 63) * t.nrep + q) * t.L + slot];
  const uint32_t nc = word_nc(w);
  for (uint32_t c = threadIdx.x; c < nc; c += blockDim.x)
    *reinterpret_cast<uint4*>(out + ao[i] + 16ull * c) =
        *reinterpret_cast<const uint4*>(a.pool + stream_byte(a.pt, a.PTS, q, inf.y + c));
}

hipError_t launch_gather_cmds(const AdminParams& a, uint32_t rid, uint64_t first, uint32_t n, const uint64_t* ao,
                              uint8_t* out, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(gather_cmds_kernel, dim3(n), dim3(256), 0, s, a, rid, first, ao, out);
  return hipGetLastError();
}

// import (one block): the view into the current state; the replica's old stream pages back to the
// free ring; a fresh stream of ceil(nch / 256) pages (the head taken by compare-and-swap, so an empty
// pool changes nothing); then every entry's ring word, info {slot crc, position} and Cmd chunks
__global__ void __launch_bounds__(256) scatter_replica_kernel(AdminParams a, uint32_t rid, const rg_replica_view* vv,
                                                              const uint64_t* words, const uint32_t* crcs,
                                                              const uint32_t* pos, const uint8_t* chunks,
                                                              uint32_t nent, uint32_t nch, uint32_t* status) {
  const TickParams& t = a.t;
  const uint32_t q = q_of(t, rid);
  const uint64_t N = t.nrep;
  const rg_replica_view& v = *vv;
  uint32_t* s32 = ((uint32_t*)(t.s32)) + q;
  uint64_t* s64 = ((uint64_t*)(t.s64)) + q;
  __shared__ uint32_t ok;
  const uint32_t np = t.P ? vpn_ceil(nch) : 0u;
  if (threadIdx.x == 0) {
    ok = 1;
    if (t.P) {
      PoolCtl* c = a.poolctl;
      unsigned long long h = c->head;
      for (;;) {  // take np ids below limit (written by earlier launches)
        if (h + np > c->limit) {
          ok = 0;
          break;
        }
        const unsigned long long seen = atomicCAS(&c->head, h, h + np);
        if (seen == h) break;
        h = seen;
      }
      if (ok) {
        const uint32_t lpg = s32[S_LPG * N], apg = s32[S_APG * N], f = vpn_diff(apg, lpg);
        uint32_t* ptq = a.pt + (uint64_t)q * a.PTS;
        const unsigned long long fb = f ? atomicAdd(&c->tail, (unsigned long long)f) : 0ull;
        for (uint32_t k = 0; k < f; ++k) a.fring[(fb + k) % a.npages] = ptq[(lpg + k) & (a.PTS - 1)];
        for (uint32_t k = 0; k < np; ++k) ptq[k & (a.PTS - 1)] = a.fring[(h + k) % a.npages];
        s32[S_HW * N] = nch;
        s32[S_LPG * N] = 0;
        s32[S_APG * N] = np;
        s32[S_NLPG * N] = 0;
      } else {
        *status = 1;
      }
    }
  }
  __syncthreads();
  if (!ok) return;
  if (threadIdx.x == 0) {
    s64[S_TERM * N] = v.term; s64[S_VOTE * N] = v.vote; s64[S_LEADER * N] = v.leader;
    s64[S_COMMITTED * N] = v.committed; s64[S_APPLIED * N] = v.applied; s64[S_LAST * N] = v.last;
    s64[S_MARKER * N] = v.marker; s64[S_MARKER_TERM * N] = v.marker_term; s64[S_SNAP_INDEX * N] = v.snap_index;
    s64[S_SNAP_TERM * N] = v.snap_term; s64[S_CAP_BASE * N] = v.cap_base; s64[S_PROCESSED * N] = v.processed;
    s64[S_LAST_TERM * N] = v.last > v.marker ? words[v.last - v.marker - 1] & TERM_MASK : v.marker_term;
    s32[S_ROLE * N] = v.role; s32[S_ETICK * N] = v.election_tick; s32[S_HTICK * N] = v.heartbeat_tick;
    s32[S_RAND_TO * N] = v.rand_timeout; s32[S_RNG_CTR * N] = v.rng_ctr; s32[S_GRANTED * N] = v.granted;
    s32[S_RESPONDED * N] = v.responded; s32[S_ACTIVE * N] = v.active; s32[S_ERR * N] = v.err;
    s32[S_DROPS * N] = v.drops;
    s32[S_MEMBERS * N] = v.members; s32[S_SNAP_MEMBERS * N] = v.snap_members; s32[S_CC_PENDING * N] = v.cc_pending;
    s64[S_CC_HI * N] = v.last;  // any imported entry may be a ConfigChange
    uint64_t* rem = ((uint64_t*)(t.rem));
    uint8_t* rst = ((uint8_t*)(t.rst));
    for (uint32_t j = 0; j < t.R; ++j) {
      rem[(0 * t.R + j) * N + q] = v.match[j];
      rem[(1 * t.R + j) * N + q] = v.next[j];
      rem[(2 * t.R + j) * N + q] = v.rsnap[j];
      rst[j * N + q] = v.rstate[j];
    }
  }
  for (uint32_t i = threadIdx.x; i < nent; i += blockDim.x) {
    const uint64_t idx = v.marker + 1 + i, slot = idx & (t.L - 1);
    const uint64_t w = words[i] & ~BANK_BIT;
    t.tr[slot * N + q] = w;
    const_cast<uint2*>(a.info)[(uint64_t)q * t.L + slot] = make_uint2((w & PAY_BIT) ? crcs[i] : 0u, pos[i]);
  }
  if (chunks)
    for (uint32_t c = threadIdx.x; c < nch; c += blockDim.x)
      *reinterpret_cast<uint4*>(a.pool + stream_byte(a.pt, a.PTS, q, c)) = reinterpret_cast<const uint4*>(chunks)[c];
}

hipError_t launch_scatter_replica(const AdminParams& a, uint32_t rid, const void* view, const uint64_t* words,
                                  const uint32_t* crcs, const uint32_t* pos, const uint8_t* chunks, uint32_t nent,
                                  uint32_t nch, uint32_t* status, hipStream_t s) {
  hipLaunchKernelGGL(scatter_replica_kernel, dim3(1), dim3(256), 0, s, a, rid, (const rg_replica_view*)view, words,
                     crcs, pos, chunks, nent, nch, status);
  return hipGetLastError();
}

// deliver: append a header to rid_src's last-tick outbox (inline terms from the sender's log)
__global__ void deliver_kernel(AdminParams a, uint32_t rid, const rg_msg_view* m, uint32_t* status) {
  const TickParams& t = a.t;
  const uint32_t g = rid / t.R, s = rid - g * t.R, q = s * t.G + g;
  const uint32_t dst = m->to - 1;
  uint32_t* cnt = ((uint32_t*)(t.cnt_in)) + ((uint64_t)s * t.R + dst) * t.G + g;
  const uint32_t k = cnt_n(*cnt);  // its class bits stay MC_ALL (0): the receiver loads every word
  if (k >= t.K) {
    *status = 1;
    return;
  }
  const uint64_t plane = (uint64_t)t.R * t.R * t.K * t.G;
  uint64_t* h = ((uint64_t*)(t.hdr_in)) + (((uint64_t)s * t.R + dst) * t.K + k) * t.G + g;
  const uint64_t* src = reinterpret_cast<const uint64_t*>(m);
  for (int w = 0; w < 8; ++w) h[w * plane] = src[w];
  if (m->type == M_REPLICATE) {  // every inline word written below: never a uniform Replicate
    h[7 * plane] = src[7] & ~(uint64_t)RG_UNIFORM;
    uint64_t* mt = ((uint64_t*)(t.mt_in)) + ((((uint64_t)s * t.R + dst) * t.K + k) * t.E) * t.G + g;
    for (uint32_t e = 0; e < m->nent; ++e) mt[(uint64_t)e * t.G] = t.tr[((m->log_index + 1 + e) & (t.L - 1)) * t.nrep + q];
  }
  *cnt = (*cnt & ~0xFFu) | (k + 1);
  *status = 0;
}

hipError_t launch_deliver(const AdminParams& a, uint32_t rid_src, const void* hdr, uint32_t* status, hipStream_t s) {
  hipLaunchKernelGGL(deliver_kernel, dim3(1), dim3(1), 0, s, a, rid_src, (const rg_msg_view*)hdr, status);
  return hipGetLastError();
}

__global__ void notify_applied_kernel(AdminParams a, const uint32_t* rids, const uint64_t* index, uint32_t n, int pass,
                                      uint32_t* bad) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const TickParams& t = a.t;
  if (rids[i] >= t.nrep) {
    atomicAdd(bad, 1u);
    return;
  }
  const uint64_t q = q_of(t, rids[i]), N = t.nrep;
  uint64_t* s64 = ((uint64_t*)(t.s64)) + q;
  if (pass == 0) {
    if (index[i] > s64[S_PROCESSED * N]) atomicAdd(bad, 1u);
  } else {
    s64[S_APPLIED * N] = index[i];
  }
}

// rg_compact: a lane per slot of the shard. Between ticks the next step's input state is
// s64; the marker moves there as a snapshot's compaction moves it at the end of a step, and the next
// step, finding it off cap_base, releases the payload stream below entry c + 1 ("Release")
__global__ void compact_kernel(AdminParams a, uint64_t group, uint64_t index, uint32_t* n) {
  const uint32_t s = threadIdx.x;
  const TickParams& t = a.t;
  if (s >= t.R || pl_rank_of(t.pl, group, s) != t.pl.rank) return;
  const uint64_t j = group / t.pl.N - t.pl.col_base, q = (uint64_t)s * t.G + j, N = t.nrep;
  uint64_t* s64 = ((uint64_t*)(t.s64)) + q;
  const uint64_t marker = s64[S_MARKER * N], snap = s64[S_SNAP_INDEX * N];
  const uint64_t c = index < snap ? index : snap;  // snap <= applied <= committed <= last: c is in the ring
  if (c <= marker) return;
  s64[S_MARKER_TERM * N] = t.tr[(c & (t.L - 1)) * N + q] & TERM_MASK;
  s64[S_MARKER * N] = c;
  atomicAdd(n, 1u);
}

hipError_t launch_compact(const AdminParams& a, uint64_t group, uint64_t index, uint32_t* n, hipStream_t s) {
  hipLaunchKernelGGL(compact_kernel, dim3(1), dim3(64), 0, s, a, group, index, n);
  return hipGetLastError();
}

hipError_t launch_notify_applied(const AdminParams& a, const uint32_t* rids, const uint64_t* index, uint32_t n,
                                 int pass, uint32_t* bad, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(notify_applied_kernel, dim3((n + 255) / 256), dim3(256), 0, s, a, rids, index, n, pass, bad);
  return hipGetLastError();
}

// ---- rg_digest (the same function as the oracle's or_digest): per replica an fmix64
// chain over its view and one over its log (marker, last], seeded by the global replica id, summed
__device__ __forceinline__ uint64_t dg_mix(uint64_t z) {
  z ^= z >> 33;
  z *= 0xFF51AFD7ED558CCDULL;
  z ^= z >> 33;
  z *= 0xC4CEB9FE1A85EC53ULL;
  z ^= z >> 33;
  return z;
}

__global__ void __launch_bounds__(256) digest_kernel(AdminParams a, unsigned long long* out) {
  const TickParams& t = a.t;
  const uint64_t N = t.nrep;
  uint64_t sa = 0, sb = 0;
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < N; q += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t s = (uint32_t)(q / t.G), g = (uint32_t)(q - (uint64_t)s * t.G);
    const uint64_t gid = pl_group(t.pl, s, g) * t.R + s;
    const uint64_t* s64 = t.s64 + q;
    const uint32_t* s32 = t.s32 + q;
    uint64_t h = dg_mix(gid + 0x9E3779B97F4A7C15ULL);
    for (uint32_t k = 0; k <= S_PROCESSED; ++k) {  // term .. processed, in rg_replica_view order
      const uint32_t row = k <= S_CAP_BASE ? k : S_PROCESSED;
      h = dg_mix(h ^ s64[row * N]);
    }
    const uint32_t rows32[13] = {S_ROLE, S_ETICK, S_HTICK, S_RAND_TO, S_RNG_CTR, S_GRANTED, S_RESPONDED, S_ACTIVE,
                                 S_ERR, S_DROPS, S_MEMBERS, S_SNAP_MEMBERS, S_CC_PENDING};
    for (uint32_t k = 0; k < 13; ++k) {
      uint32_t x = s32[rows32[k] * N];
      if (rows32[k] == S_ERR) x |= a.crc_err[q];
      h = dg_mix(h ^ x);
    }
    for (uint32_t j = 0; j < t.R; ++j) {
      h = dg_mix(h ^ t.rem[(0 * t.R + j) * N + q]);
      h = dg_mix(h ^ t.rem[(1 * t.R + j) * N + q]);
      h = dg_mix(h ^ t.rem[(2 * t.R + j) * N + q]);
      h = dg_mix(h ^ t.rst[j * N + q]);
    }
    sa += h;
    const uint64_t marker = s64[S_MARKER * N], last = s64[S_LAST * N];
    uint64_t h2 = dg_mix(gid ^ 0x5851F42D4C957F2DULL);
    for (uint64_t i = marker + 1; i <= last; ++i) {
      const uint64_t slot = i & (t.L - 1);
      const uint64_t w = t.tr[slot * N + q];
      const uint32_t type = (uint32_t)((w >> 61) & 1);
      const uint32_t len = (w & (PAY_BIT | TYPE_BIT)) ? word_len(w) : 0u;
      uint32_t crc = 0;
      if (w & PAY_BIT) crc = crc_of_cmd(a.info[((w >> 63) * N + q) * t.L + slot].x, len, t.P, a.zi);
      h2 = dg_mix(h2 ^ (w & TERM_MASK));
      h2 = dg_mix(h2 ^ ((uint64_t)type | ((uint64_t)len << 8) | ((uint64_t)crc << 32)));
    }
    sb += h2;
  }
  for (int off = 32; off > 0; off >>= 1) {
    sa += ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(sa >> 32), off, 64) << 32) | (uint32_t)__shfl_xor((int)(uint32_t)sa, off, 64);
    sb += ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(sb >> 32), off, 64) << 32) | (uint32_t)__shfl_xor((int)(uint32_t)sb, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(out, (unsigned long long)sa);
    atomicAdd(out + 1, (unsigned long long)sb);
  }
}

hipError_t launch_digest(const AdminParams& a, unsigned long long* out, hipStream_t s) {
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((a.t.nrep + 255) / 256, 4096);
  hipLaunchKernelGGL(digest_kernel, dim3(blocks), dim3(256), 0, s, a, out);
  return hipGetLastError();
}

// rg_commit_update(RG_COMMIT_APPLIED): every replica of the slot mask has applied what it was handed
// (applied = processed), one lane per replica
__global__ void applied_all_kernel(AdminParams a, uint32_t slot_mask) {
  const TickParams& t = a.t;
  const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, N = t.nrep;
  if (q >= N || !((slot_mask >> (q / t.G)) & 1u)) return;
  uint64_t* s64 = ((uint64_t*)(t.s64)) + q;
  s64[S_APPLIED * N] = s64[S_PROCESSED * N];
}

hipError_t launch_applied_all(const AdminParams& a, uint32_t slot_mask, hipStream_t s) {
  hipLaunchKernelGGL(applied_all_kernel, dim3((a.t.nrep + 255) / 256), dim3(256), 0, s, a, slot_mask);
  return hipGetLastError();
}

}  // namespace rg
