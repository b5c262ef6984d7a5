// raftgpu_bulk.hip — bulk_kernel: the payload stage (entry Cmd copy + CRC-32), one
// (wire, multi-job) variant per translation unit: the build compiles this file four times
// (-DRG_BULK_W=0/1 -DRG_BULK_MJ=0/1), each with the seven lane-group sizes.
#include <cstdlib>
#include <algorithm>
#include <type_traits>

#include "raftgpu_dev.h"

#if !defined(RG_BULK_W) || !defined(RG_BULK_MJ)
#error "compile raftgpu_bulk.hip with -DRG_BULK_W=0|1 -DRG_BULK_MJ=0|1 (raftd_amd/build.py)"
#endif

namespace rg {

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

// bulk_small_kernel's replicas (C5's load: one or two entries per replica per tick): exactly one job,
// uniform, 1..SMALL_N entries of at most P bytes each, from the sender's stream, a slab or a Cmd arena,
// and well-formed (set_job's checks for those kinds; anything else stays with bulk_kernel, which
// flags a malformed job)
constexpr uint32_t SMALL_N = 4;
__device__ __forceinline__ bool small_job(const BulkParams& p, uint32_t nj, const Job& jb, uint32_t q, uint32_t nch,
                                          bool wire) {
  if (nj != 1) return false;
  const uint32_t n = jb.meta & 0xFF, e0 = (jb.meta >> 8) & 0xFF, kind = (jb.meta >> 16) & 0xF;
  const uint32_t ncu = (jb.meta >> 21) & 0x7F;
  if (!((jb.meta >> 20) & 1u) || e0 >= n || n - e0 > SMALL_N || ncu > nch) return false;
  if (kind == SRC_RING) return jb.src < p.nrep;
  if (kind != SRC_SLAB && kind != SRC_CMD) return false;
  const uint64_t row = wire ? (uint64_t)(jb.src >> 16) * p.G + q % p.G : q % p.G;
  if ((jb.src & 0xFFFFu) >= p.nslab || row >= (wire ? p.nrep : p.G)) return false;
  if (kind == SRC_SLAB) return ncu == nch;
  return (jb.spos + (uint64_t)(n - e0) * ncu) * 16 <= p.cmd_cap;
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
#ifndef RG_TILE_SLOTMAJOR
  if constexpr (MJ) {  // a block bulk_small_kernel took whole: nothing to load (C5: every block)
    if (p.small && !p.rest[(g0 >> 6) * p.R + s]) {
      tj = TileJobs{};
      cur.m = 0;
      cur.j = 0;
      cur.njl = 0;
      return;
    }
  }
#endif
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
  bool mine = tj.nj != 0;
  if constexpr (MJ) {  // the replicas bulk_small_kernel took are done
    if (p.small && mine && small_job(p, tj.nj, tj.j0, q, p.P >> 4, p.wire_mode != 0)) mine = false;
  }
  cur.m = __ballot(mine);
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
      // the segment chain starts from the CRC's init value: raw(~0 · Z^(S·P)) ^ raw(Cmd) = the CRC before
      // its final xor, whatever the length (no per-length finalisation constant)
      uint32_t acc = 0xFFFFFFFFu;
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
      const uint32_t cr = acc ^ 0xFFFFFFFFu;
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
  // a corrupt parameter block made control skip its tick: the job tables are stale, run nothing
  if (p.poolctl->param_err) return;
  // pages freed by this tick's pool kernel become allocatable from the next tick on
  if (blockIdx.x == 0 && threadIdx.x == 0) p.poolctl->limit = p.poolctl->tail;
  if constexpr (MJ) {  // bulk_small_kernel took every replica with jobs this tick (its stamp is older)
    if (p.small && *p.rest_tick != p.tick) return;
  }
  const uint32_t shw = CRC_T_WORDS + CRC_N_WORDS + NCH * CRC_SH_STRIDE;
  for (uint32_t i = threadIdx.x; i < shw; i += blockDim.x) lds[i] = p.crc_tab[i];
  for (uint32_t i = threadIdx.x; i < CRC_ZP_WORDS; i += blockDim.x) lds[shw + i] = p.crc_tab[CRC_ZP_OFF + i];
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

// ---- bulk_small_kernel (MJ engines, before bulk_kernel): the small_job replicas, one entry per
// lane group. bulk_kernel's cursor is wave-uniform, so a one-entry job fills NCH of its 64 lanes per
// step (C5: 16 of 64 at P 256) and each job's page ids cost a scalar round trip before its payload
// load can issue. Here a wave takes a tile of 64 replicas, lists the entries of its small jobs (LDS),
// and moves EPI entries per step, each lane group with its own replica, page ids and addresses
// (vector loads), SMALL_U steps in flight.
#ifndef RG_SMALL_U
#define RG_SMALL_U 4
#endif
constexpr int SMALL_U = RG_SMALL_U;

template <int LG, bool WIRE>
__global__ void __launch_bounds__(256) bulk_small_kernel(BulkParams p, const uint32_t* __restrict__ pt) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  constexpr uint32_t NCH = 1u << LG, EPI = 64u >> LG, P = 16u << LG;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  if (p.poolctl->param_err) return;  // stale job tables (a skipped control tick): run nothing
  const uint32_t shw = CRC_T_WORDS + CRC_N_WORDS + NCH * CRC_SH_STRIDE;
  for (uint32_t i = threadIdx.x; i < shw; i += blockDim.x) lds[i] = p.crc_tab[i];
  __syncthreads();
  const uint32_t lane = lane_id(), c = lane & (NCH - 1), ei = lane >> LG, w = threadIdx.x >> 6;
  const Crc crc{lds, lds + CRC_T_WORDS, lds + CRC_T_WORDS + CRC_N_WORDS + c * CRC_SH_STRIDE, nullptr};
  uint8_t* own = reinterpret_cast<uint8_t*>(lds + shw) + w * 64 * SMALL_N;  // this wave's entry list
  const uint64_t n64 = p.nrep, L = p.L, rows = WIRE ? p.nrep : p.G, PTSM = p.PTS - 1;
  const uint32_t cols = (p.G + 63) / 64, ntiles = cols * p.R, stride = gridDim.x * (blockDim.x >> 6);
  for (uint32_t t = rfl(blockIdx.x * (blockDim.x >> 6) + w); t < ntiles; t += stride) {
    const uint32_t b = t / p.R, s = t - b * p.R, g = b * 64 + lane;
    const bool valid = g < p.G;
    const uint32_t q = s * p.G + g;
    const uint32_t nj = valid ? p.jcnt[q] : 0u;
    Job jb{};
    if (nj == 1) jb = load_job(p, q, 0);
    const bool small = valid && small_job(p, nj, jb, q, NCH, WIRE);
    // bulk_kernel skips a block of 64 groups whose replicas with jobs were all taken here
    const uint64_t left = __ballot(valid && nj != 0 && !small);
    if (lane == 0) p.rest[t] = left != 0 ? 1u : 0u;
    if (lane == 0 && left) *p.rest_tick = p.tick;  // bulk_kernel has work this tick (every writer stores the same value)
    const uint32_t e0 = (jb.meta >> 8) & 0xFF, k = small ? (jb.meta & 0xFF) - e0 : 0u;
    const uint32_t off = wave_excl_scan32(k);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)(off + k), 63);
    for (uint32_t i = 0; i < k; ++i) own[off + i] = (uint8_t)lane;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (uint32_t base = 0; base < total; base += EPI * SMALL_U) {
      u32x4 x[SMALL_U];
      uint32_t want[SMALL_U], dch[SMALL_U], it_q[SMALL_U], it_e[SMALL_U], it_dp[SMALL_U];
      uint64_t it_first[SMALL_U], it_dm[SMALL_U];
      bool act[SMALL_U], lead[SMALL_U], chk[SMALL_U];
#pragma unroll
      for (int u = 0; u < SMALL_U; ++u) {  // issue: the entry's page ids, then its payload and sender CRC
        const uint32_t it = base + u * EPI + ei;
        const bool live = it < total;
        const uint32_t l = live ? own[it] : 0u;
        const uint32_t i = it - (uint32_t)__shfl((int)off, (int)l, 64);
        const uint32_t meta = (uint32_t)__shfl((int)jb.meta, (int)l, 64), src = (uint32_t)__shfl((int)jb.src, (int)l, 64);
        const uint32_t dpos = (uint32_t)__shfl((int)jb.dpos, (int)l, 64);
        const uint64_t first = ((uint64_t)(uint32_t)__shfl((int)(jb.first >> 32), (int)l, 64) << 32) |
                               (uint32_t)__shfl((int)(uint32_t)jb.first, (int)l, 64);
        const uint64_t spos = ((uint64_t)(uint32_t)__shfl((int)(jb.spos >> 32), (int)l, 64) << 32) |
                              (uint32_t)__shfl((int)(uint32_t)jb.spos, (int)l, 64);
        const uint64_t sm = ((uint64_t)(uint32_t)__shfl((int)(jb.sm >> 32), (int)l, 64) << 32) |
                            (uint32_t)__shfl((int)(uint32_t)jb.sm, (int)l, 64);
        const uint64_t dm = ((uint64_t)(uint32_t)__shfl((int)(jb.dm >> 32), (int)l, 64) << 32) |
                            (uint32_t)__shfl((int)(uint32_t)jb.dm, (int)l, 64);
        const uint32_t ie0 = (meta >> 8) & 0xFF, kind = (meta >> 16) & 0xF, ncu = (meta >> 21) & 0x7F;
        const uint32_t e = ie0 + i, iq = s * p.G + b * 64 + l;
        const bool a = live && c < ncu;
        const bool ring = kind == SRC_RING;
        // destination: chunk dpos + i·ncu + c of this replica's stream
        const uint32_t dl = dpos + i * ncu + c;
        const uint32_t pid = a ? pt[(uint64_t)iq * p.PTS + (vpn_of(dl) & PTSM)] : 0u;
        dch[u] = pid * PAGE_CH + (dl & (PAGE_CH - 1));
        const uint8_t* sp;
        if (ring) {
          const uint32_t sl = (uint32_t)spos + e * ncu + c;
          const uint32_t sid = a ? pt[(uint64_t)src * p.PTS + (vpn_of(sl) & PTSM)] : 0u;
          sp = p.pool + (uint64_t)sid * PAGE_BYTES + ((sl & (PAGE_CH - 1)) << 4);
        } else {
          const uint32_t sl16 = src & 0xFFFFu;
          const uint64_t row = WIRE ? (uint64_t)(src >> 16) * p.G + (b * 64 + l) : (uint64_t)(b * 64 + l);
          sp = kind == SRC_CMD ? p.cmds + (uint64_t)sl16 * p.cmd_cap + 16ull * ((uint32_t)spos + i * ncu + c)
                               : p.slabs + (((uint64_t)sl16 * rows + row) * p.E + e) * P + c * 16;
        }
        const uint64_t slot = (first + e) & (L - 1);
        const uint32_t* wp = (ring && a) ? &p.info[(((sm >> e) & 1ull) * n64 + src) * L + slot].x : nullptr;
        x[u] = a ? *reinterpret_cast<const u32x4*>(sp) : u32x4{0, 0, 0, 0};
        want[u] = wp ? *wp : 0u;
        act[u] = a;
        lead[u] = live && c == 0;
        chk[u] = ring;
        it_q[u] = iq;
        it_e[u] = e;
        it_dp[u] = dpos + i * ncu;
        it_first[u] = first;
        it_dm[u] = dm;
        (void)rows;
      }
#pragma unroll
      for (int u = 0; u < SMALL_U; ++u) {  // consume: store, CRC, info word, sender-CRC check
        if (act[u]) __builtin_nontemporal_store(x[u], reinterpret_cast<u32x4*>(p.pool + (uint64_t)dch[u] * 16));
        uint32_t v = crc.raw16(make_uint4(x[u].x, x[u].y, x[u].z, x[u].w));
        if constexpr (LG > 0) v = xor_lanes<LG>(crc.shift(v));
        if (lead[u]) put_info(p, it_q[u], it_first[u], it_dm[u], it_e[u], act[u] ? (p.crc_const ^ v) : 0u, it_dp[u],
                              chk[u] && act[u], want[u]);
      }
    }
    __builtin_amdgcn_wave_barrier();  // the list is rewritten for the next tile
  }
  (void)n64;
}

static int lg_of(uint32_t P) {
  int lg = 0;
  while ((16u << lg) < P) ++lg;
  return lg;
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

template <>
hipError_t launch_bulk_t<(bool)RG_BULK_W, (bool)RG_BULK_MJ>(const BulkParams& p, const uint32_t* pt, hipStream_t s,
                                                          int grid) {
#if RG_BULK_MJ
  if (p.small) {  // the small jobs first, then bulk_kernel for the rest (it skips them)
    const uint32_t lg = (uint32_t)lg_of(p.P), nch = 1u << lg;
    const uint32_t tiles = ((p.G + 63) / 64) * p.R;
#ifdef RG_AB_SMALL_GRID  // A/B variant: workgroups per bulk-grid slot (r04: 2, 4 and 8 tie, 16 loses)
    constexpr uint32_t gmul = RG_AB_SMALL_GRID;
#else
    constexpr uint32_t gmul = 2;
#endif
    const int sg = (int)std::min<uint32_t>((tiles + 3) / 4, (uint32_t)grid * gmul);
    const int lds = (int)((CRC_T_WORDS + CRC_N_WORDS + nch * CRC_SH_STRIDE) * 4 + 4 * 64 * SMALL_N);
    hipError_t r = hipErrorInvalidValue;
    switch (lg) {
#define RG_SMALL_CASE(X) \
  case X: hipLaunchKernelGGL((bulk_small_kernel<X, (bool)RG_BULK_W>), dim3(sg), dim3(256), lds, s, p, pt); r = hipGetLastError(); break;
      RG_SMALL_CASE(0) RG_SMALL_CASE(1) RG_SMALL_CASE(2) RG_SMALL_CASE(3) RG_SMALL_CASE(4) RG_SMALL_CASE(5) RG_SMALL_CASE(6)
#undef RG_SMALL_CASE
      default: break;
    }
    if (r != hipSuccess) return r;
  }
#endif
  return with_bulk_w<(bool)RG_BULK_W, (bool)RG_BULK_MJ>(p.P, [&](auto k) {
    const uint32_t wg = p.wg_waves >= 1 && p.wg_waves <= 4 ? p.wg_waves : 4u;
    hipLaunchKernelGGL(k, dim3(grid), dim3(64 * wg), bulk_lds_bytes(p.P), s, p, pt);
    return hipGetLastError();
  });
}

template <>
int bulk_occupancy_t<(bool)RG_BULK_W, (bool)RG_BULK_MJ>(uint32_t P) {
  int n = 0;
  const hipError_t r = with_bulk_w<(bool)RG_BULK_W, (bool)RG_BULK_MJ>(P, [&](auto k) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 256, bulk_lds_bytes(P));
  });
  return (r == hipSuccess && n > 0) ? n : 1;
}

}  // namespace rg
