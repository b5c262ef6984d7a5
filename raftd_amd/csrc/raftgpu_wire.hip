// raftgpu_wire.hip — the per-tick replica-message exchange between ranks.
//
// dragonboat hands each outbound pb.Message to its transport after the step (send-after-step,
// internal/raft peer.go GetUpdate → transport); here every message a replica emitted in tick t
// to a replica on another rank travels in one batch before tick t+1, as per-rank regions the
// caller's transport moves (RCCL all-to-all over xGMI in bench.py, loopback copies in tests).
//
// A *unit* is one (sender slot s, destination slot d, column j) outbox column: up to K messages.
// Units are listed per destination rank in (s, d, j) order (host-built, identical on the sender
// and the receiver). A region for one rank is
//     [256-B header: u64 region bytes the sender's plan asked for (the fixed-capacity exchange sizes
//      the next regions on it)]
//     [u64 table: (data offset in 16-B units) << 8 | message count, one per unit, padded to 256 B]
//     [data: per message a 64-B header, then n 16-B entry records {ring word, slot crc, payload chunk
//      offset}, then the n Cmds back to back, each rounded up to 16 B — n = the entry count of a
//      Replicate, or of a forwarded Propose when P > 0 (its Cmds: records {len bits, 0, offset}); 0
//      for every other type]
// so a follower's (or a leader's, for a proposal) bulk job reads the payloads and sender CRCs
// straight out of the receive buffer. Only Cmd bytes cross xGMI (the ring word carries the length,
// raftgpu_internal.h).
//
// plan_kernel      thread per unit: 16-B units of its messages
// scan_*           exclusive scan of the unit sizes (three passes)
// pack_kernel      wave per unit: headers, records (term word + the sender's stored CRC), the Cmds
//                  copied out of the sender's payload stream (or slab / Cmd arena for a Propose)
// unpack_kernel    thread per received unit: dense remote-inbox planes (rhdr/rmt/rcnt, the layout
//                  control_kernel reads), header word 7 of a Replicate = its records' byte offset;
//                  records are checked (lengths, offsets, sizes) before anything is kept
#include "raftgpu_wire.h"

namespace rg {

__device__ __forceinline__ uint32_t wl_lane() { return __lane_id(); }

__device__ __forceinline__ void unit_decode(uint32_t u, uint32_t& s, uint32_t& d, uint32_t& j) {
  s = u >> 28;
  d = (u >> 24) & 0xF;
  j = u & 0xFFFFFF;
}

// entries a message carries on the wire: a Replicate's, and a forwarded Propose's Cmds (P > 0)
__device__ __forceinline__ uint32_t wire_entries(uint64_t w0, uint32_t P) {
  const uint32_t t = (uint32_t)(w0 & 0xFF);
  return (t == M_REPLICATE || (t == M_PROPOSE && P)) ? (uint32_t)(w0 >> 32) : 0u;
}

// payload chunks of entry e of outbox message k of column (col, j) (the sender's view)
__device__ __forceinline__ uint32_t msg_entry_nc(const WireParams& w, uint64_t col, uint32_t j, uint32_t k, uint64_t w0,
                                                 uint64_t w7, uint32_t e) {
  if ((w0 & 0xFF) == M_PROPOSE) {  // a forwarded batch: its Cmds in this replica's row of slab w7
    const uint32_t sl = (uint32_t)w7;
    if (sl >= w.nslab) return 0u;
    const uint64_t qs = (col / w.R) * w.G + j;
    return (min(w.slab_info[((uint64_t)sl * w.nrep + qs) * w.E + e].y, w.maxc) + 15u) >> 4;
  }
  const uint64_t* mtp = w.mt + ((col * w.K + k) * w.E) * w.G + j;
  const bool uni = ((uint32_t)w7 & RG_UNIFORM) != 0;
  return word_nc(mtp[uni ? 0 : (uint64_t)e * w.G]);
}

__global__ void plan_kernel(WireParams w) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= w.U) return;
  uint32_t s, d, j;
  unit_decode(w.umap[u], s, d, j);
  const uint64_t col = (uint64_t)s * w.R + d;
  const uint64_t plane = (uint64_t)w.R * w.R * w.K * w.G;
  const uint32_t c = min(cnt_n(w.cnt[col * w.G + j]), w.K);
  uint32_t sz = 0;
  for (uint32_t k = 0; k < c; ++k) {  // 16-B units: header 4, a record per entry, the Cmd chunks
    const uint64_t* h = w.hdr + (col * w.K + k) * w.G + j;
    const uint64_t w0 = h[0];
    const uint32_t n = min(wire_entries(w0, w.P), w.E);
    sz += 4u + n;
    if (n && w.P) {
      const uint64_t w7 = h[7 * plane];
      for (uint32_t e = 0; e < n; ++e) sz += msg_entry_nc(w, col, j, k, w0, w7, e);
    }
  }
  w.usize[u] = sz;
}

// ---- exclusive scan of usize[0..U) into uoff[0..U] (uoff[U] = total), 1024 elements per block
constexpr uint32_t SCAN_T = 256, SCAN_V = 4, SCAN_B = SCAN_T * SCAN_V;

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
  const uint32_t lane = wl_lane();
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, o, 64);
    const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), o, 64);
    if (lane >= o) v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}

// block-wide exclusive scan of one value per thread; returns the exclusive prefix, *total = block sum
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t* total) {
  __shared__ uint64_t wsum[SCAN_T / 64];
  const uint32_t lane = wl_lane(), wv = threadIdx.x >> 6;
  const uint64_t inc = wave_incl_scan(v);
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  uint64_t pre = 0, tot = 0;
  for (uint32_t i = 0; i < SCAN_T / 64; ++i) {
    pre += i < wv ? wsum[i] : 0;
    tot += wsum[i];
  }
  __syncthreads();
  *total = tot;
  return pre + inc - v;
}

__global__ void scan_reduce_kernel(const uint32_t* in, uint32_t n, uint64_t* bsum) {
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_B;
  uint64_t v = 0;
  for (uint32_t i = 0; i < SCAN_V; ++i) {
    const uint64_t x = base + (uint64_t)threadIdx.x * SCAN_V + i;
    v += x < n ? in[x] : 0u;
  }
  uint64_t tot;
  block_excl_scan(v, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ void scan_blocks_kernel(uint64_t* bsum, uint32_t nb) {  // one block, exclusive in place
  uint64_t carry = 0;
  for (uint32_t b0 = 0; b0 < nb; b0 += SCAN_T) {
    const uint32_t i = b0 + threadIdx.x;
    const uint64_t v = i < nb ? bsum[i] : 0;
    uint64_t tot;
    const uint64_t ex = block_excl_scan(v, &tot);
    if (i < nb) bsum[i] = carry + ex;
    carry += tot;
  }
}

__global__ void scan_apply_kernel(const uint32_t* in, uint32_t n, const uint64_t* bsum, uint64_t* out) {
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_B;
  uint32_t x[SCAN_V];
  uint64_t v = 0;
  for (uint32_t i = 0; i < SCAN_V; ++i) {
    const uint64_t k = base + (uint64_t)threadIdx.x * SCAN_V + i;
    x[i] = k < n ? in[k] : 0u;
    v += x[i];
  }
  uint64_t tot;
  uint64_t run = bsum[blockIdx.x] + block_excl_scan(v, &tot);
  for (uint32_t i = 0; i < SCAN_V; ++i) {
    const uint64_t k = base + (uint64_t)threadIdx.x * SCAN_V + i;
    if (k < n) out[k] = run;
    run += x[i];
    if (k + 1 == n) out[n] = run;
  }
}

// per-destination data sizes (16-B units) → bounds[r] = uoff[ubeg[r]], r = 0..N
__global__ void bounds_kernel(WireParams w, uint64_t* bounds) {
  const uint32_t r = threadIdx.x;
  if (r <= w.pl.N) bounds[r] = w.U ? w.uoff[w.ubeg[r]] : 0;
}

__device__ __forceinline__ uint32_t find_rank(const uint32_t* beg, uint32_t N, uint32_t u) {
  uint32_t r = 0;
  while (r + 1 < N && u >= beg[r + 1]) ++r;
  return r;
}

__device__ __forceinline__ uint64_t table_bytes(uint32_t units) { return ((uint64_t)units * 8 + 255) & ~255ull; }

__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t l) {
  // readlane returns int: widen through uint32_t, or bit 31 of the low word sign-extends over the high word
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t lane_incl_scan32(uint32_t v) {
  const uint32_t lane = wl_lane();
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)v, o, 64);
    if (lane >= o) v += y;
  }
  return v;
}

__global__ void __launch_bounds__(256) pack_kernel(WireParams w) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint32_t lane = wl_lane();
  const uint32_t u = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  if (u >= w.U) return;
  const uint32_t r = find_rank(w.ubeg, w.pl.N, u);
  const uint32_t u0 = w.ubeg[r], nu = w.ubeg[r + 1] - u0;
  uint8_t* region = w.send + w.send_region[r];
  const uint64_t off16 = w.uoff[u] - w.uoff[u0];
  uint32_t s, d, j;
  unit_decode(w.umap[u], s, d, j);
  const uint64_t col = (uint64_t)s * w.R + d, qs = (uint64_t)s * w.G + j, n64 = w.nrep;
  const uint64_t plane = (uint64_t)w.R * w.R * w.K * w.G;
  uint32_t c = cnt_n(w.cnt[col * w.G + j]);
  if (c > w.K) {
    RG_OOB("RG_BOUNDS pack u=%u s=%u d=%u j=%u cnt=%u > K\n", u, s, d, j, c);
    c = 0;
  }
  const uint64_t tb = table_bytes(nu);
  if (u == u0 && lane == 0) {  // the header: the bytes this region needs (the receiver sizes the next ones on it)
    const uint64_t need = 256 + tb + (w.uoff[w.ubeg[r + 1]] - w.uoff[u0]) * 16;
    reinterpret_cast<uint64_t*>(region)[0] = need;
    if (w.sneed) w.sneed[r] = need;
  }
  // fixed-capacity exchange: a unit whose data would end past the region is dropped whole (its table
  // entry says no messages; Raft retries, as with a message lost in transit), and counted
  const uint64_t cap = w.send_cap[r];
  if (cap && 256 + tb + (off16 + w.usize[u]) * 16 > cap) {
    if (lane == 0) {
      reinterpret_cast<uint64_t*>(region + 256)[u - u0] = off16 << 8;
      if (c && w.drops) atomicAdd(w.drops, (unsigned long long)c);
    }
    return;
  }
  if (lane == 0) reinterpret_cast<uint64_t*>(region + 256)[u - u0] = (off16 << 8) | c;
  uint8_t* out = region + 256 + tb + off16 * 16;
  const uint32_t P = w.P;
  for (uint32_t k = 0; k < c; ++k) {
    const uint64_t* hp = w.hdr + (col * w.K + k) * w.G + j;
    const uint64_t hv = lane < 8 ? hp[lane * plane] : 0;
    if (lane < 8) reinterpret_cast<uint64_t*>(out)[lane] = hv;
    const uint64_t w0 = rl64(hv, 0), li = rl64(hv, 3), w7 = rl64(hv, 7);
    const bool prop = (w0 & 0xFF) == M_PROPOSE;
    // a uniform Replicate: one inline word for every entry; expanded into n records on the wire
    const uint64_t est = (w0 & 0xFF) == M_REPLICATE && ((uint32_t)w7 & RG_UNIFORM) ? 0ull : (uint64_t)w.G;
    uint32_t n = wire_entries(w0, P);
    if (n > w.E) {  // plan_kernel sized the region with the same n: only reachable on corrupt state
      RG_OOB("RG_BOUNDS pack u=%u k=%u n=%u > E\n", u, k, n);
      n = 0;
    }
    // a forwarded Propose: its Cmds are in this replica's row of slab w7 (the bytes its tick staged)
    const uint32_t sl = (uint32_t)w7;
    const bool slab_ok = prop && sl < w.nslab;
    const uint64_t se0 = ((uint64_t)sl * n64 + qs) * w.E;
    const uint64_t* mtp = w.mt + ((col * w.K + k) * w.E) * w.G + j;
    // lane e: entry e's record and where its Cmd is (sender stream position / slab / arena chunk)
    uint64_t word = 0;
    uint32_t crc = 0, nc = 0, sp = 0;
    bool syn = false;
    if (lane < n) {
      if (prop) {
        const uint2 inf = slab_ok ? w.slab_info[se0 + lane] : make_uint2(0u, 0u);
        word = len_bits(min(inf.y, w.maxc));
        syn = (inf.x & SYN_OFF) != 0;
        sp = inf.x & ~SYN_OFF;
      } else {
        word = mtp[(uint64_t)lane * est];
        const uint64_t slot = (li + 1 + lane) & (w.L - 1);
        const uint2 inf = w.info[((word >> 63) * n64 + qs) * w.L + slot];
        crc = (word & PAY_BIT) ? inf.x : 0u;
        sp = inf.y;
      }
      nc = P ? word_nc(word) : 0u;
    }
    const uint32_t inc = lane_incl_scan32(nc), total = __builtin_amdgcn_readlane(inc, 63);
    if (lane < n)
      *reinterpret_cast<u32x4*>(out + 64 + 16 * lane) = u32x4{(uint32_t)word, (uint32_t)(word >> 32), crc, inc - nc};
    uint8_t* po = out + 64 + 16ull * n;
    for (uint32_t t = lane; t < ((total + 63) & ~63u); t += 64) {
      uint32_t lo = 0;  // the entry of chunk t: first lane with inc > t
#pragma unroll
      for (uint32_t step = 32; step; step >>= 1) {
        const uint32_t v = (uint32_t)__shfl((int)inc, (int)(lo + step - 1), 64);
        if (v <= t) lo += step;
      }
      const uint32_t le = lo < 64 ? lo : 63;
      // every lane takes part in the permute: a lane masked off by a branch supplies no data, and a
      // reader of it (lane lo - 1 with its own lo = 0) would get 0
      const uint32_t exl = (uint32_t)__shfl((int)inc, (int)(lo ? lo - 1 : 0), 64);
      const uint32_t ex = lo ? exl : 0u;
      const uint32_t spl = (uint32_t)__shfl((int)sp, (int)le, 64);
      const bool synl = __shfl((int)syn, (int)le, 64) != 0;
      if (t < total) {
        const uint32_t ch = t - ex;
        const uint8_t* src = !prop ? w.pool + stream_byte(w.pt, w.PTS, (uint32_t)qs, spl + ch)
                             : synl ? w.slabs + (se0 + le) * P + 16ull * ch
                                    : w.cmds + (uint64_t)sl * w.cmd_cap + 16ull * (spl + ch);
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src));
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(po + 16ull * t));
      }
    }
    out += 64 + 16ull * (n + total);
  }
}

__device__ __forceinline__ bool cc_valid(uint32_t cc, uint32_t R) {  // a ConfigChange descriptor (or none)
  const uint32_t op = cc >> 4, sl = cc & 0xF;
  return cc == 0 || ((op == CC_ADD || op == CC_REMOVE) && sl >= 1 && sl <= R && cc <= 0x2Fu);
}

__global__ void unpack_kernel(WireParams w) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= w.RU) return;
  const uint32_t r = find_rank(w.rbeg, w.pl.N, u);
  const uint32_t u0 = w.rbeg[r], nu = w.rbeg[r + 1] - u0;
  const uint8_t* region = w.recv + w.recv_region[r];
  if (u == u0 && w.rneed) {  // the need the sender's plan put in the header, checked: it comes from another process
    // and sizes this link's capacity on both ends, so a bad one is reported (~0: the host fails the next
    // rg_wire_plan_fixed) rather than fed to the capacity rule, where the two ends would then disagree
    const uint64_t need = reinterpret_cast<const uint64_t*>(region)[0];
    const uint64_t lo = 256 + ((nu * 8ull + 255) & ~255ull);
    const uint64_t hi = lo + (uint64_t)nu * w.K * (64 + (uint64_t)w.E * (16 + ((w.maxc + 15ull) & ~15ull)));
    w.rneed[r] = (need >= lo && need <= hi && !(need & 15)) ? need : ~0ull;
  }
  const uint64_t tv = reinterpret_cast<const uint64_t*>(region + 256)[u - u0];
  uint32_t c = (uint32_t)(tv & 0xFF);
  const uint64_t rend = r + 1 < w.pl.N ? w.recv_region[r + 1] : w.recv_total;
  uint32_t s, d, j;
  unit_decode(w.rmap[u], s, d, j);
  const uint64_t col = (uint64_t)s * w.R + d;
  const uint64_t plane = (uint64_t)w.R * w.R * w.K * w.G;
  if (c > w.K || (tv >> 8) > (rend >> 4)) {  // count beyond K, or a data offset beyond the buffer
    RG_OOB("RG_BOUNDS unpack u=%u r=%u s=%u d=%u j=%u cnt=%u off16=%llu\n", u, r, s, d, j, c,
           (unsigned long long)(tv >> 8));
    c = 0;
  }
  const uint8_t* in = region + 256 + table_bytes(nu) + (c ? (tv >> 8) * 16 : 0);
  // malformed data (a count or size beyond the region): keep only the messages before it
  uint32_t k = 0, cls = 0;  // cls: the kept messages' classes (cnt_cls), as the sender's count plane has them
  for (; k < c; ++k) {
    if ((uint64_t)(in - w.recv) + 64 > rend) {
      RG_OOB("RG_BOUNDS unpack u=%u k=%u header beyond region end %llu\n", u, k, (unsigned long long)rend);
      break;
    }
    const uint64_t* h = reinterpret_cast<const uint64_t*>(in);
    const uint64_t w0 = h[0];
    const uint32_t type = (uint32_t)(w0 & 0xFF), n = wire_entries(w0, w.P);
    // exchange data comes from another process: keep a message only if this plane can carry it —
    // a known type, from the unit's sender slot s to its destination slot d, at most E entries (a
    // Propose 1..E with a valid ConfigChange descriptor or none), inside the region; the unit's
    // messages from the first bad one on are dropped
    const bool known = type == M_NOOP || type == M_PROPOSE || type == M_REPLICATE || type == M_REPLICATE_RESP ||
                       type == M_REQUEST_VOTE || type == M_REQUEST_VOTE_RESP || type == M_INSTALL_SNAPSHOT ||
                       type == M_HEARTBEAT || type == M_HEARTBEAT_RESP || type == M_READ_INDEX ||
                       type == M_READ_INDEX_RESP;
    const uint32_t from = (uint32_t)(w0 >> 8) & 0xFF, to = (uint32_t)(w0 >> 16) & 0xFF, nent = (uint32_t)(w0 >> 32);
    // terms fit the ring word's 36-bit field (a replica never makes a larger one: rg_import_replica
    // refuses it, a campaign at the limit is refused, RG_ERR_TERM_LIMIT)
    const bool terms_ok = h[1] <= TERM_MASK &&
                          (h[2] <= TERM_MASK || !(type == M_REPLICATE || type == M_REQUEST_VOTE || type == M_INSTALL_SNAPSHOT));
    if (!known || !terms_ok || from != s + 1 || to != d + 1 || n > w.E ||
        (type == M_PROPOSE && (nent < 1 || nent > w.E || !cc_valid((uint32_t)h[6], w.R))) ||
        (uint64_t)(in - w.recv) + 64 + (uint64_t)n * 16 > rend) {
      RG_OOB("RG_BOUNDS unpack u=%u k=%u type=%u from=%u to=%u n=%u region end %llu\n", u, k, type, from, to, n,
             (unsigned long long)rend);
      break;
    }
    // every entry record: an application entry's length <= max_cmd_bytes with the payload bit exactly
    // when non-zero, a ConfigChange no payload and a descriptor; Cmd offsets back to back from 0
    bool sane = true, same = n > 0;
    uint32_t tot = 0;
    for (uint32_t e = 0; e < n; ++e) {
      const uint64_t rw = h[8 + 2 * e];
      const uint32_t ln = word_len(rw), ofs = (uint32_t)(h[9 + 2 * e] >> 32);
      sane = sane && ((rw & TYPE_BIT) ? !(rw & PAY_BIT) && ln <= 0x2Fu
                                      : ln <= w.maxc && ((rw & PAY_BIT) != 0) == (ln != 0)) &&
             ofs == tot;
      same = same && rw == h[8] && !(rw & TYPE_BIT);
      tot += word_nc(rw);
    }
    if (!sane || (uint64_t)(in - w.recv) + 64 + 16ull * (n + tot) > rend) {
      RG_OOB("RG_BOUNDS unpack u=%u k=%u: a bad entry record or Cmds beyond the region\n", u, k);
      break;
    }
    uint64_t* ho = w.rhdr + (col * w.K + k) * w.G + j;
    for (int x = 0; x < 7; ++x) ho[x * plane] = h[x];
    if (type == M_PROPOSE) ho[4 * plane] = tot;  // its Cmds' stream chunks (the capacity rule's input)
    // entries: word 7 = their records' offset (16-B aligned), | RG_UNIFORM for a Replicate whose records
    // all hold one application ring word (the control kernel's fast path appends it as one uniform job)
    ho[7 * plane] = n ? (uint64_t)(in + 64 - w.recv) | (type == M_REPLICATE && same ? (uint64_t)RG_UNIFORM : 0ull)
                      : h[7];
    uint64_t* mo = w.rmt + ((col * w.K + k) * w.E) * w.G + j;  // inline ring words (a Propose: length bits)
    for (uint32_t e = 0; e < n; ++e) mo[(uint64_t)e * w.G] = h[8 + 2 * e] & (type == M_PROPOSE ? ~TERM_MASK & ~BANK_BIT & ~TYPE_BIT : ~0ull);
    in += 64 + 16ull * (n + tot);
    if (k < 4) cls |= msg_class(type, nent) << (2 * k);
  }
  w.rcnt[col * w.G + j] = k | (cls << 8);
}

hipError_t launch_wire_plan(const WireParams& w, uint64_t* bounds, hipStream_t st) {
  if (w.U) {
    hipLaunchKernelGGL(plan_kernel, dim3((w.U + 255) / 256), dim3(256), 0, st, w);
    const uint32_t nb = (w.U + SCAN_B - 1) / SCAN_B;
    hipLaunchKernelGGL(scan_reduce_kernel, dim3(nb), dim3(SCAN_T), 0, st, w.usize, w.U, w.bsum);
    hipLaunchKernelGGL(scan_blocks_kernel, dim3(1), dim3(SCAN_T), 0, st, w.bsum, nb);
    hipLaunchKernelGGL(scan_apply_kernel, dim3(nb), dim3(SCAN_T), 0, st, w.usize, w.U, w.bsum, w.uoff);
  }
  hipLaunchKernelGGL(bounds_kernel, dim3(1), dim3(64), 0, st, w, bounds);
  return hipGetLastError();
}

hipError_t launch_scan_u32(const uint32_t* in, uint32_t n, uint64_t* bsum, uint64_t* out, hipStream_t st) {
  if (!n) return hipMemsetAsync(out, 0, 8, st);
  const uint32_t nb = (n + SCAN_B - 1) / SCAN_B;
  hipLaunchKernelGGL(scan_reduce_kernel, dim3(nb), dim3(SCAN_T), 0, st, in, n, bsum);
  hipLaunchKernelGGL(scan_blocks_kernel, dim3(1), dim3(SCAN_T), 0, st, bsum, nb);
  hipLaunchKernelGGL(scan_apply_kernel, dim3(nb), dim3(SCAN_T), 0, st, in, n, bsum, out);
  return hipGetLastError();
}

hipError_t launch_wire_pack(const WireParams& w, hipStream_t st) {
  if (!w.U) return hipSuccess;
  hipLaunchKernelGGL(pack_kernel, dim3((w.U + 3) / 4), dim3(256), 0, st, w);
  return hipGetLastError();
}

hipError_t launch_wire_unpack(const WireParams& w, hipStream_t st) {
  if (!w.RU) return hipSuccess;
  hipLaunchKernelGGL(unpack_kernel, dim3((w.RU + 255) / 256), dim3(256), 0, st, w);
  return hipGetLastError();
}

}  // namespace rg
