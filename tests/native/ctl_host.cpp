// ctl_host.cpp — TEST HARNESS: runs the engine's control step (raftgpu_control.h, the body of
// control_kernel<R>) on the CPU over host copies of the device's structure-of-arrays layout, so
// the exact GPU control code can be checked against the oracle and run under AddressSanitizer
// without a GPU. The bulk (payload/CRC) kernel is not emulated beyond what the control step reads
// back: each written entry's stream position (its info word) and the pool kernel's page bookkeeping
// (S_LPG / S_APG); entries carry terms/types only.
#define RG_FN inline
#include "../../raftd_amd/csrc/raftgpu_control.h"
#include "../../include/raftgpu.h"

#include <cstring>
#include <vector>

using namespace rg;

struct Host {
  int fast = 0;             // ch_set_fast: 1 / 2 the fast-path step first (2: its latency build), the full
                            // step for a lane it hands off; 3 the full step's SLIM build (control_slow_kernel)
  uint64_t slow_lanes = 0;  // lanes the fast path handed off (all ticks)
  rg_config c;
  uint32_t nrep, J;
  std::vector<uint64_t> s64, rem, tr, hdr[2], mt[2], job64;  // state rows in place, as on the device
  std::vector<uint2> info;        // [2 banks][nrep][L] {crc (0 here), stream position}
  uint32_t PTS = 16;
  std::vector<uint32_t> s32, cnt[2], job32, jcnt;
  std::vector<uint8_t> rst;
  uint64_t violations = 0;  // ch_violations: state invariants broken after a step, or a fast step that
                            // handed off after writing state (its in-place rows must be untouched)
  std::vector<uint2> slab_info;  // [nslab][G][E] {0, len}: synthetic Cmds are P bytes; ch_propose sets lengths
  std::vector<uint64_t> rdst;     // ReadIndex state rows
  std::vector<uint64_t> feed;     // the step's hand-off words (feed_word), as on the device
  std::vector<uint64_t> rd;       // rg_read_index staging: ctx per (group, slot), 0 = none
  bool rd_staged = false;
  std::vector<uint8_t> pt;        // rg_propose staging: target slot, count, non-empty mask per group
  std::vector<uint32_t> pc;
  std::vector<uint64_t> hm;
  std::vector<uint2> pcmd;  // {stream chunks | contiguous << 31, arena chunk}: chunk counts only here
  bool staged = false;
  std::vector<uint16_t> cc;  // membership change staging: slot | descriptor << 8
  bool cc_staged = false;
  uint64_t t = 0;
  // wire_all (rg_config.wire_all): every plane is remote, so the step reads the remote inbox planes
  // (rhdr / rmt / rcnt) that unpack_kernel writes on the device; emulate_wire fills them from the last
  // step's outbox as pack_kernel + unpack_kernel would (the control step's view of the wire)
  bool wire = false;
  std::vector<uint64_t> rhdr, rmt;
  std::vector<uint32_t> rcnt;
};

static TickParams params(Host* h) {
  TickParams p{};
  const rg_config& c = h->c;
  p.G = c.groups; p.R = c.replicas; p.nrep = h->nrep; p.L = c.log_capacity; p.P = c.payload_bytes;
  p.E = c.max_entries_per_msg; p.K = c.max_msgs_per_pair; p.nslab = c.num_slabs; p.J = h->J;
  p.ET = c.election_rtt; p.HT = c.heartbeat_rtt; p.CQ = c.check_quorum; p.SE = c.snapshot_entries;
  p.CO = c.compaction_overhead; p.drop_ppm = c.drop_ppm; p.seed = c.seed; p.tick = h->t;
  p.AF = c.apply_feedback;
  p.PTS = h->PTS;
  p.JS = c.join_slots;
  p.IM = c.initial_members;
  p.info = h->info.data();
  p.pl = make_placement(1, 0, h->wire ? 1u : 0u);  // one rank: every plane local, or (wire_all) remote
  p.wire = h->wire ? 1u : 0u;  // a wire engine's slab rows are per replica
  if (h->wire) {
    p.rhdr = h->rhdr.data();
    p.rmt = h->rmt.data();
    p.rcnt = h->rcnt.data();
  }
  const int a = (int)(h->t & 1), b = a ^ 1;
  p.s64 = h->s64.data(); p.s32 = h->s32.data(); p.rem = h->rem.data(); p.rst = h->rst.data();
  p.tr = h->tr.data();
  p.hdr_in = h->hdr[b].data(); p.hdr_out = h->hdr[a].data();
  p.mt_in = h->mt[b].data(); p.mt_out = h->mt[a].data();
  p.cnt_in = h->cnt[b].data(); p.cnt_out = h->cnt[a].data();
  p.job64 = h->job64.data(); p.job32 = h->job32.data(); p.jcnt = h->jcnt.data();
  p.slab_info = h->slab_info.data();
  p.rdst = h->rdst.data();
  p.feed = h->feed.data();
  return p;
}

static uint32_t qof(Host* h, uint32_t rid) {
  const uint32_t g = rid / h->c.replicas, s = rid % h->c.replicas;
  return s * h->c.groups + g;
}

extern "C" {

void* ch_create(const rg_config* c) {
  Host* h = new Host();
  h->c = *c;
  h->nrep = c->groups * c->replicas;
  h->J = (c->replicas - 1) * c->max_msgs_per_pair + 2;
  const size_t n = h->nrep, L = c->log_capacity, R = c->replicas, K = c->max_msgs_per_pair,
               E = c->max_entries_per_msg, G = c->groups, J = h->J;
  h->s64.assign(S64_ROWS * n, 0);
  h->s32.assign(S32_ROWS * n, 0);
  h->rem.assign(3 * R * n, 0);
  h->rst.assign(R * n, 0);
  for (int b = 0; b < 2; ++b) {
    h->hdr[b].assign(8 * R * R * K * G, 0);
    h->mt[b].assign(R * R * K * E * G, 0);
    h->cnt[b].assign(R * R * G, 0);
  }
  h->tr.assign(L * n, 0);
  h->info.assign(2 * L * n, make_uint2(0u, 0u));
  {  // stream_pages as rg_create sizes it
    const uint64_t full = ((uint64_t)L * ((c->payload_bytes + 15) & ~15u) + PAGE_BYTES - 1) / PAGE_BYTES;
    uint32_t pts = 16;
    while (pts < 2 * full) pts <<= 1;
    h->PTS = c->payload_bytes ? (c->stream_pages ? c->stream_pages : pts) : 1;
  }
  h->job64.assign(J64_ROWS * J * n, 0);
  h->job32.assign(J32_ROWS * J * n, 0);
  h->jcnt.assign(n, 0);
  h->feed.assign(n, 0);
  h->wire = c->wire_all != 0;
  h->slab_info.assign((size_t)c->num_slabs * (h->wire ? n : G) * E, make_uint2(0u, c->payload_bytes));
  if (h->wire) {
    h->rhdr.assign(8 * R * R * K * G, 0);
    h->rmt.assign(R * R * K * E * G, 0);
    h->rcnt.assign(R * R * G, 0);
  }
  h->rdst.assign((size_t)RD_ROWS * n, 0);
  h->rd.assign(n, 0);
  h->pt.assign(G, 0xFF);
  h->pc.assign(G, 0);
  h->hm.assign(G, 0);
  h->pcmd.assign(G, make_uint2(0u, 0u));
  h->cc.assign(G, 0);
  return h;
}

void ch_destroy(void* hh) { delete (Host*)hh; }
// the fast path (control_fast_kernel + control_slow_kernel on the device): on = 1
void ch_set_fast(void* hh, int on) { ((Host*)hh)->fast = on; }
uint64_t ch_slow_lanes(void* hh) { return ((Host*)hh)->slow_lanes; }
uint64_t ch_violations(void* hh) { return ((Host*)hh)->violations; }

// placement math of raftgpu_internal.h, for the CPU cross-check with raftd_amd/cluster.py
uint64_t ch_pl_group(uint32_t N, uint32_t rank, uint32_t s, uint32_t j) {
  return pl_group(make_placement(N, rank, 0), s, j);
}
uint32_t ch_pl_off(uint32_t N, uint32_t s, uint32_t d, uint32_t j) { return pl_off(make_placement(N, 0, 0), s, d, j); }

void ch_bootstrap(void* hh) {  // = bootstrap_kernel
  Host* h = (Host*)hh;
  h->t = 0;
  const uint32_t R = h->c.replicas, JS = h->c.join_slots;
  const uint64_t n = h->nrep;
  for (int b = 0; b < 2; ++b) std::fill(h->cnt[b].begin(), h->cnt[b].end(), 0u);
  const uint32_t im = (h->c.initial_members ? h->c.initial_members : (1u << R) - 1u) & ~JS;
  for (uint32_t q = 0; q < n; ++q) {
    const uint32_t s = q / h->c.groups, g = q - s * h->c.groups;
    const bool joining = (JS >> s) & 1u;
    const uint64_t last = joining ? 0 : R;
    for (uint32_t f = 0; f < S64_ROWS; ++f) h->s64[f * n + q] = 0;
    for (uint32_t f = 0; f < S32_ROWS; ++f) h->s32[f * n + q] = 0;
    h->s64[S_TERM * n + q] = joining ? 0 : 1;
    h->s64[S_LAST * n + q] = last;
    h->s64[S_LAST_TERM * n + q] = last ? 1 : 0;
    h->s64[S_COMMITTED * n + q] = last;
    h->s64[S_CC_HI * n + q] = last;
    h->s32[S_RNG_CTR * n + q] = 1;
    h->s32[S_MEMBERS * n + q] = joining ? 0u : im;
    h->s32[S_SNAP_MEMBERS * n + q] = joining ? 0u : im;
    const uint64_t key = ((uint64_t)g << 32) | ((uint64_t)s << 24) | 1ull;
    h->s32[S_RAND_TO * n + q] = h->c.election_rtt + (uint32_t)(mix64(h->c.seed ^ mix64(key)) % h->c.election_rtt);
    for (uint32_t j = 0; j < R; ++j) {
      h->rem[(0 * R + j) * n + q] = 0;
      h->rem[(1 * R + j) * n + q] = last + 1;
      h->rem[(2 * R + j) * n + q] = 0;
      h->rst[j * n + q] = RETRY;
    }
    for (uint32_t i = 1; i <= last; ++i) {
      const uint32_t cc = ((im >> (i - 1)) & 1u) ? (CC_ADD << 4 | i) : 0u;
      h->tr[(i & (h->c.log_capacity - 1)) * n + q] = 1ull | TYPE_BIT | cc_bits(cc);
      h->info[(uint64_t)q * h->c.log_capacity + (i & (h->c.log_capacity - 1))] = make_uint2(0u, 0u);
    }
  }
}

// what the pool and bulk kernels leave behind that a later control step reads: the pages held
// ([S_LPG, S_APG)) and every written entry's info word {0, stream position} (positions back to back
// from the job's J_DPOS, as the bulk kernel lays them out)
static void after_step(Host* h, const TickParams& p) {
  const uint64_t n = h->nrep, L = h->c.log_capacity, JN = (uint64_t)h->J * n;
  uint32_t* so = const_cast<uint32_t*>(p.s32);
  for (uint64_t q = 0; q < n; ++q) {
    so[S_LPG * n + q] = so[S_NLPG * n + q];
    so[S_APG * n + q] = vpn_ceil(so[S_HW * n + q]);
    for (uint32_t j = 0; j < p.jcnt[q]; ++j) {
      const uint64_t jq = (uint64_t)j * n + q, first = p.job64[J_FIRST * JN + jq], dm = p.job64[J_DMASK * JN + jq];
      const uint32_t meta = p.job32[J_META * JN + jq], nn = meta & 0xFF, e0 = (meta >> 8) & 0xFF;
      uint32_t pos = p.job32[J_DPOS * JN + jq];
      for (uint32_t e = e0; e < nn; ++e) {
        const uint64_t slot = (first + e) & (L - 1);
        h->info[(((dm >> e) & 1ull) * n + q) * L + slot] = make_uint2(0u, pos);
        pos += word_nc(h->tr[slot * n + q]);
      }
    }
  }
}
// What pack_kernel + the transfer + unpack_kernel leave for the next step's control kernel when every
// plane is remote (raftgpu_wire.hip): the remote inbox planes. Headers are copied; a Replicate's inline
// words expanded per entry (a uniform one's single word repeated); a forwarded Propose's words are its
// Cmds' length bits from the forwarder's slab row and its header word 4 their stream chunks; word 7 of a
// message with entries = a 16-B aligned offset of its records in one receive buffer, | RG_UNIFORM for a
// Replicate whose records all hold one application ring word. The payload bytes themselves (the bulk
// kernel's input) are not emulated.
static void emulate_wire(Host* h, const TickParams& p) {
  const uint64_t G = p.G, R = p.R, K = p.K, E = p.E, n64 = p.nrep, plane = R * R * K * G;
  const uint32_t maxc = h->c.max_cmd_bytes ? h->c.max_cmd_bytes : h->c.payload_bytes;
  uint64_t off = 256;
  for (uint64_t col = 0; col < R * R; ++col) {
    const uint64_t s = col / R, d = col % R;
    for (uint64_t j = 0; j < G; ++j) {
      uint32_t c = s == d ? 0u : cnt_n(p.cnt_in[col * G + j]);
      if (c > K) c = 0;
      uint32_t cls = 0;  // the kept messages' classes, as unpack_kernel recomputes them
      for (uint32_t k = 0; k < c && k < 4; ++k) {
        const uint64_t w0k = p.hdr_in[(col * K + k) * G + j];
        cls |= msg_class((uint32_t)(w0k & 0xFF), (uint32_t)(w0k >> 32)) << (2 * k);
      }
      h->rcnt[col * G + j] = c | (cls << 8);
      for (uint32_t k = 0; k < c; ++k) {
        const uint64_t* hs = p.hdr_in + (col * K + k) * G + j;
        uint64_t* ho = h->rhdr.data() + (col * K + k) * G + j;
        const uint64_t w0 = hs[0], w7 = hs[7 * plane];
        const uint32_t type = (uint32_t)(w0 & 0xFF);
        const uint32_t n = (type == M_REPLICATE || (type == M_PROPOSE && p.P)) ? (uint32_t)(w0 >> 32) : 0u;
        const bool uni = type == M_REPLICATE && ((uint32_t)w7 & RG_UNIFORM);
        const uint64_t* mts = p.mt_in + ((col * K + k) * E) * G + j;
        uint64_t* mto = h->rmt.data() + ((col * K + k) * E) * G + j;
        bool same = n > 0;
        uint64_t first = 0;
        uint32_t tot = 0;
        for (uint32_t e = 0; e < n; ++e) {
          uint64_t word;
          if (type == M_PROPOSE) {
            const uint32_t sl = (uint32_t)w7, len = h->slab_info[(((uint64_t)sl * n64) + s * G + j) * E + e].y;
            word = len_bits(len < maxc ? len : maxc);
          } else {
            word = mts[(uni ? 0 : (uint64_t)e) * G];
          }
          if (e == 0) first = word;
          same = same && word == first && !(word & TYPE_BIT);
          tot += word_nc(word);
          mto[(uint64_t)e * G] = type == M_PROPOSE ? (word & ~TERM_MASK & ~BANK_BIT & ~TYPE_BIT) : word;
        }
        for (int x = 0; x < 7; ++x) ho[x * plane] = hs[x * plane];
        if (type == M_PROPOSE) ho[4 * plane] = tot;
        ho[7 * plane] = n ? (off | (type == M_REPLICATE && same ? (uint64_t)RG_UNIFORM : 0ull)) : w7;
        off += 64 + 16ull * (n + tot);
      }
    }
  }
}

// the product's fast step (control_fast_kernel / control_fastfb_kernel): the role-specialised Ctl,
// lean (fast mode 1, the large-engine kernel) or the latency build (fast mode 2, small engines)
extern "C++" {
template <int R, int ROLE, bool LAT>
static bool fast_role(const TickParams& p, uint32_t q) {
  Ctl<R, true, ROLE, LAT> f(p, q);
  f.run();
  return f.aborted;
}
// replica q's state rows (the in-place state a handed-off fast step must leave untouched)
struct LaneRows {
  uint64_t v[S64_ROWS + S32_ROWS + 4 * RG_MAX_REPLICAS];
  uint32_t n = 0;
  bool operator!=(const LaneRows& o) const { return n != o.n || memcmp(v, o.v, n * 8) != 0; }
};
template <class H>
static void lane_state(H* h, uint32_t q, LaneRows& o) {
  const uint64_t n = h->nrep, R = h->c.replicas;
  o.n = 0;
  for (uint32_t f = 0; f < S64_ROWS; ++f) o.v[o.n++] = h->s64[f * n + q];
  for (uint32_t f = 0; f < S32_ROWS; ++f) o.v[o.n++] = h->s32[f * n + q];
  for (uint32_t j = 0; j < 3 * R; ++j) o.v[o.n++] = h->rem[j * n + q];
  for (uint32_t j = 0; j < R; ++j) o.v[o.n++] = h->rst[j * n + q];
}
template <int R, class H>
static bool fast_step(H* h, const TickParams& p, uint32_t q) {
  const bool lead = p.s32[(uint64_t)S_ROLE * p.nrep + q] == LEADER;
  LaneRows before, after;
  lane_state(h, q, before);
  bool ab;
  if (h->fast == 2) ab = lead ? fast_role<R, LEADER, true>(p, q) : fast_role<R, FOLLOWER, true>(p, q);
  else ab = lead ? fast_role<R, LEADER, false>(p, q) : fast_role<R, FOLLOWER, false>(p, q);
  if (ab) {  // the full step re-runs it from these rows
    lane_state(h, q, after);
    if (after != before) h->violations++;
  }
  return ab;
}
// After every step: S_LAST_TERM caches term(last) (marker_term on an empty log), the pool's
// bookkeeping left S_NLPG = S_LPG (the fast step's in-place store skips an unchanged S_NLPG), and a remote's
// snapshot index is 0 outside the SNAPSHOT state (the fast step neither reads nor writes it)
template <class H>
static void check_invariants(H* h) {
  const uint64_t n = h->nrep, R = h->c.replicas, L = h->c.log_capacity;
  for (uint64_t q = 0; q < n; ++q) {
    const uint64_t last = h->s64[S_LAST * n + q], marker = h->s64[S_MARKER * n + q];
    const uint64_t want = last > marker ? h->tr[(last & (L - 1)) * n + q] & TERM_MASK : h->s64[S_MARKER_TERM * n + q];
    if (h->s64[S_LAST_TERM * n + q] != want) h->violations++;
    if (h->s32[S_NLPG * n + q] != h->s32[S_LPG * n + q]) h->violations++;
    for (uint64_t j = 0; j < R; ++j)
      if (h->rst[j * n + q] != SNAPSHOT && h->rem[(2 * R + j) * n + q] != 0) h->violations++;
  }
}
}  // extern "C++"


int ch_tick(void* hh, const rg_tick_input* in) {
  Host* h = (Host*)hh;
  TickParams p = params(h);
  if (in) {
    p.flags = in->flags;
    p.prop_target = in->prop_target;
    p.prop_count = in->prop_count;
    p.campaign = in->campaign;
    p.isolate = in->isolate;
  }
  if (h->staged) {
    p.prop_target = h->pt.data();
    p.prop_count = h->pc.data();
    p.prop_hmask = h->hm.data();
    p.prop_cmd = h->pcmd.data();
  }
  if (h->cc_staged) p.cc_in = h->cc.data();
  if (h->rd_staged) p.read_ctx = h->rd.data();
  if (h->wire) emulate_wire(h, p);
  for (uint32_t q = 0; q < h->nrep; ++q) {
    switch (h->c.replicas) {
#define RG_CASE(r)                                  \
  case r: {                                         \
    bool full = true;                               \
    if (h->fast == 1 || h->fast == 2) {             \
      full = fast_step<r>(h, p, q);                 \
      h->slow_lanes += full;                        \
    }                                               \
    if (full && h->fast == 3) {                     \
      Ctl<r, false, -1, false, true> c(p, q);       \
      c.run();                                      \
    } else if (full) {                              \
      Ctl<r> c(p, q);                               \
      c.run();                                      \
    }                                               \
    break;                                          \
  }
      RG_CASE(1) RG_CASE(2) RG_CASE(3) RG_CASE(4) RG_CASE(5) RG_CASE(6) RG_CASE(7) RG_CASE(8)
#undef RG_CASE
      default: return -1;
    }
  }
  after_step(h, p);
  check_invariants(h);
  h->t++;
  if (h->staged) {
    std::fill(h->pt.begin(), h->pt.end(), 0xFF);
    std::fill(h->pc.begin(), h->pc.end(), 0u);
    std::fill(h->hm.begin(), h->hm.end(), 0ull);
    std::fill(h->pcmd.begin(), h->pcmd.end(), make_uint2(0u, 0u));
    h->staged = false;
  }
  if (h->cc_staged) {
    std::fill(h->cc.begin(), h->cc.end(), (uint16_t)0);
    h->cc_staged = false;
  }
  if (h->rd_staged) {
    std::fill(h->rd.begin(), h->rd.end(), 0ull);
    h->rd_staged = false;
  }
  return 0;
}

// = rg_read_index's staging (global replica id g·R + s; the caller validates)
void ch_read_index(void* hh, uint32_t rid, uint64_t ctx) {
  Host* h = (Host*)hh;
  h->rd[rid] = ctx;
  h->rd_staged = true;
}
// the reads replica rid made ready in the last tick (rdst rows, as read_count / read_gather_kernel)
int ch_read_ready(void* hh, uint32_t rid, uint64_t* ctx, uint64_t* index, uint32_t cap) {
  Host* h = (Host*)hh;
  const uint64_t n = h->nrep, q = qof(h, rid);
  if (h->rdst[RD_TICK * n + q] != h->t) return 0;
  const uint32_t k = (uint32_t)h->rdst[RD_N * n + q];
  for (uint32_t i = 0; i < k && i < cap; ++i) {
    ctx[i] = h->rdst[(RD_CTX + i) * n + q];
    index[i] = h->rdst[(RD_INDEX + i) * n + q];
  }
  return (int)k;
}

// = rg_config_change's staging (no validation beyond one change per group)
int ch_config_change(void* hh, uint32_t group, uint32_t slot, uint32_t op, uint32_t target) {
  Host* h = (Host*)hh;
  if (h->cc[group]) return -3;
  h->cc[group] = (uint16_t)(slot | ((op << 4 | (target + 1)) << 8));
  h->cc_staged = true;
  return 0;
}

// = rg_propose's staging (lengths only: the bulk kernel is not emulated); no validation
int ch_propose(void* hh, const rg_proposal* props, uint64_t n, const uint32_t* lens) {
  Host* h = (Host*)hh;
  const uint64_t E = h->c.max_entries_per_msg, slab = h->t % h->c.num_slabs, P = h->c.payload_bytes;
  for (uint64_t i = 0; i < n; ++i) {
    const rg_proposal& b = props[i];
    for (uint32_t x = 0; x < b.count; ++x) {
      const uint32_t at = h->pc[b.group] + x, ln = lens[b.first + x];
      if (ln && P) h->hm[b.group] |= 1ull << at;
      const uint64_t row = h->wire ? (uint64_t)b.slot * h->c.groups + b.group : b.group;  // wire: per replica
      h->slab_info[(slab * (h->wire ? h->nrep : h->c.groups) + row) * E + at] = make_uint2(0u, ln);
      if (P) h->pcmd[b.group].x += (ln + 15) / 16;  // not contiguous: the bulk kernel is not emulated
    }
    h->pt[b.group] = (uint8_t)b.slot;
    h->pc[b.group] += b.count;
  }
  h->staged = n > 0;
  return 0;
}

// = notify_applied_kernel's second pass
int ch_notify_applied(void* hh, uint32_t rid, uint64_t index) {
  Host* h = (Host*)hh;
  const uint64_t q = qof(h, rid), N = h->nrep;
  uint64_t* s64 = h->s64.data() + q;
  if (index > s64[S_PROCESSED * N]) return -1;
  s64[S_APPLIED * N] = index;
  return 0;
}

int ch_read_replica(void* hh, uint32_t rid, rg_replica_view* v) {
  Host* h = (Host*)hh;
  const uint32_t q = qof(h, rid);
  const uint64_t N = h->nrep;
  const uint64_t* s64 = h->s64.data() + q;
  const uint32_t* s32 = h->s32.data() + q;
  memset(v, 0, sizeof *v);
  v->term = s64[S_TERM * N]; v->vote = s64[S_VOTE * N]; v->leader = s64[S_LEADER * N];
  v->committed = s64[S_COMMITTED * N]; v->applied = s64[S_APPLIED * N]; v->last = s64[S_LAST * N];
  v->marker = s64[S_MARKER * N]; v->marker_term = s64[S_MARKER_TERM * N]; v->snap_index = s64[S_SNAP_INDEX * N];
  v->snap_term = s64[S_SNAP_TERM * N]; v->cap_base = s64[S_CAP_BASE * N]; v->processed = s64[S_PROCESSED * N];
  v->role = s32[S_ROLE * N]; v->election_tick = s32[S_ETICK * N]; v->heartbeat_tick = s32[S_HTICK * N];
  v->rand_timeout = s32[S_RAND_TO * N]; v->rng_ctr = s32[S_RNG_CTR * N]; v->granted = s32[S_GRANTED * N];
  v->responded = s32[S_RESPONDED * N]; v->active = s32[S_ACTIVE * N]; v->err = s32[S_ERR * N];
  v->drops = s32[S_DROPS * N];
  v->members = s32[S_MEMBERS * N]; v->snap_members = s32[S_SNAP_MEMBERS * N]; v->cc_pending = s32[S_CC_PENDING * N];
  const uint32_t R = h->c.replicas;
  for (uint32_t j = 0; j < R; ++j) {
    v->match[j] = h->rem[(0 * R + j) * N + q];
    v->next[j] = h->rem[(1 * R + j) * N + q];
    v->rsnap[j] = h->rem[(2 * R + j) * N + q];
    v->rstate[j] = h->rst[j * N + q];
  }
  return 0;
}

int ch_read_msgs(void* hh, uint32_t rid, uint32_t dst, rg_msg_view* out, uint32_t cap, uint64_t* terms) {
  Host* h = (Host*)hh;
  TickParams t = params(h);
  const uint32_t g = rid / t.R, s = rid % t.R;
  const uint64_t plane = (uint64_t)t.R * t.R * t.K * t.G;
  const uint32_t cnt = cnt_n(t.cnt_in[((uint64_t)s * t.R + dst) * t.G + g]);
  for (uint32_t k = 0; k < cnt && k < cap; ++k) {
    const uint64_t* hp = t.hdr_in + (((uint64_t)s * t.R + dst) * t.K + k) * t.G + g;
    uint64_t w[8];
    const uint32_t wm = hdr_words((uint32_t)(hp[0] & 0xFF), (uint32_t)(hp[0] >> 32));  // the words it carries
    for (int i = 0; i < 8; ++i) w[i] = (wm >> i) & 1u ? hp[i * plane] : 0ull;
    const bool uni = (w[0] & 0xFF) == M_REPLICATE && ((uint32_t)w[7] & RG_UNIFORM);  // shown expanded
    if (uni) {
      w[7] &= ~(uint64_t)RG_UNIFORM;
      w[5] = 0;  // its Cmds' stream position
    }
    if ((w[0] & 0xFF) == M_PROPOSE) w[4] = 0;  // its batch's stream layout
    memcpy(&out[k], w, 64);
    const uint64_t* mt = t.mt_in + ((((uint64_t)s * t.R + dst) * t.K + k) * t.E) * t.G + g;
    const uint32_t n = (uint32_t)(w[0] >> 32);
    for (uint32_t e = 0; e < t.E; ++e)
      terms[(uint64_t)k * t.E + e] =
          ((w[0] & 0xFF) == M_REPLICATE && e < n) ? (mt[uni ? 0 : (uint64_t)e * t.G] & TERM_MASK) : 0;
  }
  return (int)cnt;
}

// term-ring words (term | type<<61 | pay<<62 | bank<<63) of entries first..first+n-1
int ch_read_words(void* hh, uint32_t rid, uint64_t first, uint32_t n, uint64_t* out) {
  Host* h = (Host*)hh;
  const uint32_t q = qof(h, rid);
  for (uint32_t i = 0; i < n; ++i) out[i] = h->tr[((first + i) & (h->c.log_capacity - 1)) * h->nrep + q];
  return 0;
}

int ch_import(void* hh, uint32_t rid, const rg_replica_view* v, const uint64_t* terms, const uint32_t* types,
              int with_payload, const uint32_t* lens) {
  Host* h = (Host*)hh;
  const uint32_t q = qof(h, rid);
  const uint64_t N = h->nrep;
  uint64_t* s64 = h->s64.data() + q;
  uint32_t* s32 = h->s32.data() + q;
  s64[S_TERM * N] = v->term; s64[S_VOTE * N] = v->vote; s64[S_LEADER * N] = v->leader;
  s64[S_COMMITTED * N] = v->committed; s64[S_APPLIED * N] = v->applied; s64[S_LAST * N] = v->last;
  s64[S_MARKER * N] = v->marker; s64[S_MARKER_TERM * N] = v->marker_term; s64[S_SNAP_INDEX * N] = v->snap_index;
  s64[S_SNAP_TERM * N] = v->snap_term; s64[S_CAP_BASE * N] = v->cap_base; s64[S_PROCESSED * N] = v->processed;
  s64[S_LAST_TERM * N] = v->last > v->marker ? terms[v->last - v->marker - 1] & TERM_MASK : v->marker_term;
  h->feed[q] = 0;  // nothing to apply, persist or report until it steps (rg_import_replica)
  s32[S_ROLE * N] = v->role; s32[S_ETICK * N] = v->election_tick; s32[S_HTICK * N] = v->heartbeat_tick;
  s32[S_RAND_TO * N] = v->rand_timeout; s32[S_RNG_CTR * N] = v->rng_ctr; s32[S_GRANTED * N] = v->granted;
  s32[S_RESPONDED * N] = v->responded; s32[S_ACTIVE * N] = v->active; s32[S_ERR * N] = v->err;
  s32[S_DROPS * N] = v->drops;
  s32[S_MEMBERS * N] = v->members; s32[S_SNAP_MEMBERS * N] = v->snap_members; s32[S_CC_PENDING * N] = v->cc_pending;
  s64[S_CC_HI * N] = v->last;  // any imported entry may be a ConfigChange
  const uint32_t R = h->c.replicas;
  for (uint32_t j = 0; j < R; ++j) {
    h->rem[(0 * R + j) * N + q] = v->match[j];
    h->rem[(1 * R + j) * N + q] = v->next[j];
    h->rem[(2 * R + j) * N + q] = v->rsnap[j];
    h->rst[j * N + q] = v->rstate[j];
  }
  uint32_t pos = 0;  // a fresh payload stream from position 0 (rg_import_replica)
  for (uint64_t i = v->marker + 1; i <= v->last; ++i) {
    const uint64_t k = i - v->marker - 1;
    const uint32_t ty = types ? types[k] & 0xFFu : 0;
    const bool hp = with_payload && h->c.payload_bytes && ty == 0 && !(types && (types[k] & 0x100u));
    const uint32_t ln = lens ? lens[k] : h->c.payload_bytes;
    const uint64_t w = (terms[k] & TERM_MASK) | (ty ? TYPE_BIT : 0) | (ty ? cc_bits(lens ? lens[k] : 0) : hp ? len_bits(ln) : 0);
    h->tr[(i & (h->c.log_capacity - 1)) * N + q] = w;
    h->info[(uint64_t)q * h->c.log_capacity + (i & (h->c.log_capacity - 1))] = make_uint2(0u, pos);
    pos += word_nc(w);
  }
  s32[S_HW * N] = pos;
  s32[S_LPG * N] = 0;
  s32[S_APG * N] = vpn_ceil(pos);
  s32[S_NLPG * N] = 0;
  return 0;
}

int ch_deliver(void* hh, uint32_t rid, const rg_msg_view* m) {  // = deliver_kernel
  Host* h = (Host*)hh;
  TickParams t = params(h);
  const uint32_t g = rid / t.R, s = rid % t.R, q = s * t.G + g;
  const uint32_t dst = m->to - 1;
  uint32_t* cnt = const_cast<uint32_t*>(t.cnt_in) + ((uint64_t)s * t.R + dst) * t.G + g;
  const uint32_t k = cnt_n(*cnt);  // its class bits stay MC_ALL (0): the receiver loads every word
  if (k >= t.K) return -3;
  rg_msg_view mm = *m;
  if (mm.from == 0) mm.from = (uint8_t)(s + 1);
  const uint64_t plane = (uint64_t)t.R * t.R * t.K * t.G;
  uint64_t* hp = const_cast<uint64_t*>(t.hdr_in) + (((uint64_t)s * t.R + dst) * t.K + k) * t.G + g;
  uint64_t w[8];
  memcpy(w, &mm, 64);
  for (int i = 0; i < 8; ++i) hp[i * plane] = w[i];
  if (mm.type == M_REPLICATE) {
    uint64_t* mt = const_cast<uint64_t*>(t.mt_in) + ((((uint64_t)s * t.R + dst) * t.K + k) * t.E) * t.G + g;
    for (uint32_t e = 0; e < mm.nent; ++e) mt[(uint64_t)e * t.G] = t.tr[((mm.log_index + 1 + e) & (t.L - 1)) * t.nrep + q];
  }
  *cnt = (*cnt & ~0xFFu) | (k + 1);
  return 0;
}

// replica rid's hand-off word of the last step, decoded as rg_get_update's kernels decode it:
// {first index applied, restored index (0: none), took a snapshot, persist (entries written or the
// hard state changed), lowest index written (~0: none)}
int ch_feed(void* hh, uint32_t rid, uint64_t* out) {
  Host* h = (Host*)hh;
  if (rid >= h->nrep) return -1;
  const uint32_t q = qof(h, rid);
  const uint64_t n = h->nrep, f = h->feed[q], processed = h->s64[S_PROCESSED * n + q], last = h->s64[S_LAST * n + q];
  out[0] = feed_apply_lo(f, processed);
  out[1] = feed_restored_at(f, processed);
  out[2] = (f & FEED_TAKEN) ? 1 : 0;
  out[3] = (f & FEED_PERSIST) ? 1 : 0;
  out[4] = feed_persist_lo(f, last);
  return 0;
}

}  // extern "C"
