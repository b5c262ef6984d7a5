// raftgpu_engine.cpp — host runtime behind the C-ABI in include/raftgpu.h.
//
// Owns the device-resident replica table, builds the CRC tables, and launches
// the tick kernel. The product path has no CPU fallback: every rg_tick runs the HIP kernel and
// an engine cannot be created without a GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/raftgpu.h"
#include "raftgpu_internal.h"

using namespace rg;

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                                   \
  do {                                                                                              \
    hipError_t _e = (x);                                                                            \
    if (_e != hipSuccess) return fail(RG_EHIP, std::string(#x) + ": " + hipGetErrorString(_e));     \
  } while (0)

struct rg_engine {
  rg_config c{};
  uint32_t nrep = 0;
  hipStream_t own = nullptr, stream = nullptr;
  RepState* st[2] = {nullptr, nullptr};
  uint64_t* term_ring = nullptr;
  uint2* info = nullptr;
  uint8_t* pay = nullptr;
  MsgHdr* hdr[2] = {nullptr, nullptr};
  uint64_t* mt[2] = {nullptr, nullptr};
  uint32_t* cnt[2] = {nullptr, nullptr};
  uint8_t* slabs = nullptr;
  uint32_t* crc_tab = nullptr;
  uint32_t crc_const = 0;
  uint8_t* d_prop_target = nullptr;
  uint32_t* d_prop_count = nullptr;
  uint8_t* d_campaign = nullptr;
  uint8_t* d_isolate = nullptr;
  unsigned long long* d_sum = nullptr;
  uint64_t t = 0;
  int grid = 0;
  uint64_t bytes = 0;
  std::vector<void*> allocs;
  uint32_t T0[256];
};

// ---------------------------------------------------------------- CRC-32/IEEE tables
static void build_crc(rg_engine* e, std::vector<uint32_t>& tab) {
  uint32_t* T0 = e->T0;
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
    T0[b] = c;
  }
  auto Z = [&](uint32_t x) { return T0[x & 0xFF] ^ (x >> 8); };  // one zero byte
  auto Zn = [&](uint32_t x, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) x = Z(x);
    return x;
  };
  tab.assign(CRC_T_WORDS + CRC_S_WORDS, 0);
  for (uint32_t k = 0; k < 16; ++k)
    for (uint32_t b = 0; b < 256; ++b) tab[k * 256 + b] = Zn(T0[b], k);
  for (uint32_t j = 0; j < 6; ++j)
    for (uint32_t q = 0; q < 4; ++q)
      for (uint32_t b = 0; b < 256; ++b) tab[CRC_T_WORDS + j * 1024 + q * 256 + b] = Zn(b << (8 * q), 16u << j);
  e->crc_const = Zn(0xFFFFFFFFu, e->c.payload_bytes) ^ 0xFFFFFFFFu;
}

static uint32_t host_crc(const rg_engine* e, const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = e->T0[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

template <class T>
static int dalloc(rg_engine* e, T** p, uint64_t bytes) {
  if (bytes == 0) bytes = 16;
  hipError_t r = hipMalloc((void**)p, bytes);
  if (r != hipSuccess) {
    return fail(RG_ENOMEM, "hipMalloc(" + std::to_string(bytes) + " B) failed: " + hipGetErrorString(r));
  }
  e->allocs.push_back(*p);
  e->bytes += bytes;
  return RG_OK;
}

static bool pow2(uint32_t x) { return x && !(x & (x - 1)); }

static TickParams params(rg_engine* e) {
  TickParams p{};
  const rg_config& c = e->c;
  p.G = c.groups;
  p.R = c.replicas;
  p.nrep = e->nrep;
  p.L = c.log_capacity;
  p.P = c.payload_bytes;
  p.E = c.max_entries_per_msg;
  p.K = c.max_msgs_per_pair;
  p.nslab = c.num_slabs;
  p.ET = c.election_rtt;
  p.HT = c.heartbeat_rtt;
  p.CQ = c.check_quorum;
  p.SE = c.snapshot_entries;
  p.CO = c.compaction_overhead;
  p.drop_ppm = c.drop_ppm;
  p.crc_const = e->crc_const;
  p.seed = c.seed;
  p.tick = e->t;
  p.st_in = e->st[e->t & 1];
  p.st_out = e->st[(e->t + 1) & 1];
  p.term_ring = e->term_ring;
  p.info = e->info;
  p.pay = e->pay;
  p.hdr_in = e->hdr[(e->t + 1) & 1];
  p.hdr_out = e->hdr[e->t & 1];
  p.mt_in = e->mt[(e->t + 1) & 1];
  p.mt_out = e->mt[e->t & 1];
  p.cnt_in = e->cnt[(e->t + 1) & 1];
  p.cnt_out = e->cnt[e->t & 1];
  p.slabs = e->slabs;
  p.crc_tab = e->crc_tab;
  return p;
}

extern "C" {

const char* rg_last_error(void) { return g_err.c_str(); }

int rg_create(const rg_config* cfg, rg_engine** out) {
  if (!cfg || !out) return fail(RG_EINVAL, "null argument");
  const rg_config& c = *cfg;
  if (c.groups < 1 || c.replicas < 1 || c.replicas > RG_MAX_REPLICAS) return fail(RG_EINVAL, "groups/replicas");
  if (!pow2(c.log_capacity) || c.log_capacity < 16) return fail(RG_EINVAL, "log_capacity must be a power of two >= 16");
  if (c.payload_bytes && (!pow2(c.payload_bytes) || c.payload_bytes < 16 || c.payload_bytes > 1024))
    return fail(RG_EINVAL, "payload_bytes must be 0 or a power of two in [16, 1024]");
  if (c.max_entries_per_msg < 1 || c.max_entries_per_msg > 64) return fail(RG_EINVAL, "max_entries_per_msg in 1..64");
  if (c.max_msgs_per_pair < 1 || c.max_msgs_per_pair > 16) return fail(RG_EINVAL, "max_msgs_per_pair in 1..16");
  if (c.num_slabs < 2 || c.election_rtt < 1 || c.heartbeat_rtt < 1) return fail(RG_EINVAL, "num_slabs/rtt");
  if ((uint64_t)c.groups * c.replicas > 0xFFFFFFFFull / 2) return fail(RG_EINVAL, "too many replicas");
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (ndev <= 0 || c.device < 0 || c.device >= ndev) return fail(RG_EINVAL, "no such HIP device");
  HIPCHK(hipSetDevice(c.device));

  rg_engine* e = new rg_engine();
  e->c = c;
  e->nrep = c.groups * c.replicas;
  const uint64_t n = e->nrep, L = c.log_capacity, P = c.payload_bytes, R = c.replicas, K = c.max_msgs_per_pair,
                 E = c.max_entries_per_msg;
  int rc = RG_OK;
  for (int b = 0; b < 2 && rc == RG_OK; ++b) {
    rc = dalloc(e, &e->st[b], n * sizeof(RepState));
    if (rc == RG_OK) rc = dalloc(e, &e->hdr[b], n * R * K * sizeof(MsgHdr));
    if (rc == RG_OK) rc = dalloc(e, &e->mt[b], n * R * K * E * sizeof(uint64_t));
    if (rc == RG_OK) rc = dalloc(e, &e->cnt[b], n * R * sizeof(uint32_t));
  }
  if (rc == RG_OK) rc = dalloc(e, &e->term_ring, n * L * sizeof(uint64_t));
  if (rc == RG_OK) rc = dalloc(e, &e->info, 2 * n * L * sizeof(uint2));
  if (rc == RG_OK) rc = dalloc(e, &e->pay, 2 * n * L * P);
  if (rc == RG_OK) rc = dalloc(e, &e->slabs, (uint64_t)c.num_slabs * c.groups * E * P);
  if (rc == RG_OK) rc = dalloc(e, &e->crc_tab, (CRC_T_WORDS + CRC_S_WORDS) * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->d_prop_target, c.groups);
  if (rc == RG_OK) rc = dalloc(e, &e->d_prop_count, c.groups * 4ull);
  if (rc == RG_OK) rc = dalloc(e, &e->d_campaign, n);
  if (rc == RG_OK) rc = dalloc(e, &e->d_isolate, n);
  if (rc == RG_OK) rc = dalloc(e, &e->d_sum, 64);
  if (rc != RG_OK) {
    std::string msg = g_err;
    rg_destroy(e);
    return fail(rc, msg);
  }
  if (hipStreamCreateWithFlags(&e->own, hipStreamNonBlocking) != hipSuccess) {
    rg_destroy(e);
    return fail(RG_EHIP, "hipStreamCreate");
  }
  e->stream = e->own;
  std::vector<uint32_t> tab;
  build_crc(e, tab);
  if (hipMemcpy(e->crc_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    rg_destroy(e);
    return fail(RG_EHIP, "crc table upload");
  }
  // grid: one wave per replica, 4 waves per 256-thread workgroup
  e->grid = (int)((n + 3) / 4);
  *out = e;
  return RG_OK;
}

void rg_destroy(rg_engine* e) {
  if (!e) return;
  if (e->own) {
    (void)hipStreamSynchronize(e->own);
    (void)hipStreamDestroy(e->own);
  }
  for (void* p : e->allocs) (void)hipFree(p);
  delete e;
}

uint64_t rg_device_bytes(const rg_engine* e) { return e ? e->bytes : 0; }
uint64_t rg_tick_count(const rg_engine* e) { return e ? e->t : 0; }

int rg_set_stream(rg_engine* e, void* stream) {
  if (!e) return fail(RG_EINVAL, "null engine");
  e->stream = stream ? (hipStream_t)stream : e->own;
  return RG_OK;
}

int rg_sync(rg_engine* e) {
  if (!e) return fail(RG_EINVAL, "null engine");
  HIPCHK(hipStreamSynchronize(e->stream));
  return RG_OK;
}

int rg_bootstrap(rg_engine* e) {
  if (!e) return fail(RG_EINVAL, "null engine");
  HIPCHK(hipSetDevice(e->c.device));
  e->t = 0;
  for (int b = 0; b < 2; ++b) {
    HIPCHK(hipMemsetAsync(e->cnt[b], 0, (uint64_t)e->nrep * e->c.replicas * 4, e->stream));
  }
  TickParams p = params(e);
  p.st_out = e->st[0];
  HIPCHK(launch_bootstrap(p, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return RG_OK;
}

int rg_fill_slabs(rg_engine* e) {
  if (!e) return fail(RG_EINVAL, "null engine");
  HIPCHK(launch_fill_slabs(e->slabs, e->c.num_slabs, e->c.groups, e->c.max_entries_per_msg, e->c.payload_bytes,
                           e->c.seed, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return RG_OK;
}

static int tick_impl(rg_engine* e, const rg_tick_input* in, bool device_ptrs) {
  TickParams p = params(e);
  if (in) {
    p.flags = in->flags;
    if (device_ptrs) {
      p.prop_target = in->prop_target;
      p.prop_count = in->prop_count;
      p.campaign = in->campaign;
      p.isolate = in->isolate;
    } else {
      const uint64_t G = e->c.groups, n = e->nrep;
      if (in->prop_target) {
        if (!in->prop_count) return fail(RG_EINVAL, "prop_target without prop_count");
        for (uint64_t g = 0; g < G; ++g)
          if (in->prop_target[g] != 0xFF && in->prop_count[g] > e->c.max_entries_per_msg)
            return fail(RG_EINVAL, "proposal batch larger than max_entries_per_msg");
        HIPCHK(hipMemcpyAsync(e->d_prop_target, in->prop_target, G, hipMemcpyHostToDevice, e->stream));
        HIPCHK(hipMemcpyAsync(e->d_prop_count, in->prop_count, G * 4, hipMemcpyHostToDevice, e->stream));
        p.prop_target = e->d_prop_target;
        p.prop_count = e->d_prop_count;
      }
      if (in->campaign) {
        HIPCHK(hipMemcpyAsync(e->d_campaign, in->campaign, n, hipMemcpyHostToDevice, e->stream));
        p.campaign = e->d_campaign;
      }
      if (in->isolate) {
        HIPCHK(hipMemcpyAsync(e->d_isolate, in->isolate, n, hipMemcpyHostToDevice, e->stream));
        p.isolate = e->d_isolate;
      }
    }
  }
  HIPCHK(launch_tick(p, e->stream, e->grid));
  e->t++;
  if (!device_ptrs && in) HIPCHK(hipStreamSynchronize(e->stream));  // host buffers may be reused
  return RG_OK;
}

int rg_tick(rg_engine* e, const rg_tick_input* in) {
  if (!e) return fail(RG_EINVAL, "null engine");
  return tick_impl(e, in, false);
}

int rg_tick_device(rg_engine* e, const rg_tick_input* in) {
  if (!e) return fail(RG_EINVAL, "null engine");
  return tick_impl(e, in, true);
}

static void to_view(const RepState& s, rg_replica_view* v) {
  memset(v, 0, sizeof *v);
  v->term = s.term; v->vote = s.vote; v->leader = s.leader; v->committed = s.committed; v->applied = s.applied;
  v->last = s.last; v->marker = s.marker; v->marker_term = s.marker_term; v->snap_index = s.snap_index;
  v->snap_term = s.snap_term; v->cap_base = s.cap_base;
  v->role = s.role; v->election_tick = s.etick; v->heartbeat_tick = s.htick; v->rand_timeout = s.rand_to;
  v->rng_ctr = s.rng_ctr; v->granted = s.granted; v->responded = s.responded; v->active = s.active;
  v->err = s.err; v->drops = s.drops;
  for (int k = 0; k < RG_MAX_REPLICAS; ++k) {
    v->match[k] = s.match[k];
    v->next[k] = s.next[k];
    v->rsnap[k] = s.rsnap[k];
    v->rstate[k] = s.rstate[k];
  }
}

int rg_read_replicas(rg_engine* e, uint32_t first, uint32_t n, rg_replica_view* out) {
  if (!e || !out || (uint64_t)first + n > e->nrep) return fail(RG_EINVAL, "rg_read_replicas range");
  std::vector<RepState> buf(n);
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipMemcpy(buf.data(), e->st[e->t & 1] + first, n * sizeof(RepState), hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < n; ++i) {
    to_view(buf[i], &out[i]);
    for (uint32_t k = e->c.replicas; k < RG_MAX_REPLICAS; ++k) {
      out[i].match[k] = out[i].next[k] = out[i].rsnap[k] = 0;
      out[i].rstate[k] = 0;
    }
  }
  return RG_OK;
}

int rg_read_msgs(rg_engine* e, uint32_t rid, uint32_t dst, rg_msg_view* out, uint32_t cap, uint64_t* terms) {
  if (!e || rid >= e->nrep || dst >= e->c.replicas) return fail(RG_EINVAL, "rg_read_msgs range");
  const uint32_t R = e->c.replicas, K = e->c.max_msgs_per_pair, E = e->c.max_entries_per_msg;
  const int ob = (int)((e->t + 1) & 1);
  HIPCHK(hipStreamSynchronize(e->stream));
  uint32_t n = 0;
  HIPCHK(hipMemcpy(&n, e->cnt[ob] + (uint64_t)rid * R + dst, 4, hipMemcpyDeviceToHost));
  uint32_t m = std::min(n, cap);
  if (m && out) {
    static_assert(sizeof(rg_msg_view) == sizeof(MsgHdr), "msg view");
    HIPCHK(hipMemcpy(out, e->hdr[ob] + ((uint64_t)rid * R + dst) * K, m * sizeof(MsgHdr), hipMemcpyDeviceToHost));
  }
  if (m && terms) {
    HIPCHK(hipMemcpy(terms, e->mt[ob] + ((uint64_t)rid * R + dst) * K * E, (uint64_t)m * E * 8,
                     hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < (uint64_t)m * E; ++i) terms[i] &= TERM_MASK;
  }
  return (int)n;
}

int rg_read_entries(rg_engine* e, uint32_t rid, uint64_t first, uint32_t n, rg_entry_view* out, uint8_t* payload) {
  if (!e || rid >= e->nrep || !out) return fail(RG_EINVAL, "rg_read_entries args");
  rg_replica_view v;
  int rc = rg_read_replicas(e, rid, 1, &v);
  if (rc) return rc;
  if (n == 0) return RG_OK;
  if (first <= v.marker || first + n - 1 > v.last) return fail(RG_EINVAL, "index outside (marker, last]");
  const uint64_t L = e->c.log_capacity, P = e->c.payload_bytes;
  for (uint32_t k = 0; k < n; ++k) {
    uint64_t idx = first + k, slot = idx & (L - 1);
    uint64_t tw = 0;
    uint2 inf;
    HIPCHK(hipMemcpy(&tw, e->term_ring + (uint64_t)rid * L + slot, 8, hipMemcpyDeviceToHost));
    uint64_t bank = tw >> 63;
    HIPCHK(hipMemcpy(&inf, e->info + (bank * e->nrep + rid) * L + slot, 8, hipMemcpyDeviceToHost));
    out[k].term = tw & TERM_MASK;
    out[k].type = inf.y >> 24;
    out[k].len = inf.y & 0xFFFFFF;
    out[k].crc = inf.x;
    out[k].bank = (uint32_t)bank;
    if (payload && P && out[k].len)
      HIPCHK(hipMemcpy(payload + (uint64_t)k * P, e->pay + ((bank * e->nrep + rid) * L + slot) * P, out[k].len,
                       hipMemcpyDeviceToHost));
  }
  return RG_OK;
}

int rg_import_replica(rg_engine* e, uint32_t rid, const rg_replica_view* v, const uint64_t* terms,
                      const uint32_t* types, const uint8_t* payloads) {
  if (!e || !v || rid >= e->nrep) return fail(RG_EINVAL, "rg_import_replica args");
  const uint64_t L = e->c.log_capacity, P = e->c.payload_bytes;
  if (v->last < v->marker || v->last - v->marker > L) return fail(RG_EINVAL, "log longer than the ring");
  HIPCHK(hipStreamSynchronize(e->stream));
  RepState s{};
  s.term = v->term; s.vote = v->vote; s.leader = v->leader; s.committed = v->committed; s.applied = v->applied;
  s.last = v->last; s.marker = v->marker; s.marker_term = v->marker_term; s.snap_index = v->snap_index;
  s.snap_term = v->snap_term; s.cap_base = v->cap_base;
  s.role = v->role; s.etick = v->election_tick; s.htick = v->heartbeat_tick; s.rand_to = v->rand_timeout;
  s.rng_ctr = v->rng_ctr; s.granted = v->granted; s.responded = v->responded; s.active = v->active;
  s.err = v->err; s.drops = v->drops;
  for (int k = 0; k < RG_MAX_REPLICAS; ++k) {
    s.match[k] = v->match[k];
    s.next[k] = v->next[k];
    s.rsnap[k] = v->rsnap[k];
    s.rstate[k] = v->rstate[k];
  }
  HIPCHK(hipMemcpy(e->st[e->t & 1] + rid, &s, sizeof s, hipMemcpyHostToDevice));
  for (uint64_t i = v->marker + 1; i <= v->last; ++i) {
    uint64_t k = i - v->marker - 1, slot = i & (L - 1);
    uint64_t tw = terms[k] & TERM_MASK;
    uint32_t type = types ? types[k] : RG_ENTRY_APPLICATION;
    uint32_t len = 0, crc = 0;
    if (payloads && P && type == RG_ENTRY_APPLICATION) {
      len = (uint32_t)P;
      crc = host_crc(e, payloads + k * P, P);
      HIPCHK(hipMemcpy(e->pay + ((uint64_t)rid * L + slot) * P, payloads + k * P, P, hipMemcpyHostToDevice));
    }
    uint2 inf = make_uint2(crc, (type << 24) | len);
    HIPCHK(hipMemcpy(e->term_ring + (uint64_t)rid * L + slot, &tw, 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->info + (uint64_t)rid * L + slot, &inf, 8, hipMemcpyHostToDevice));
  }
  return RG_OK;
}

int rg_deliver(rg_engine* e, uint32_t rid_src, const rg_msg_view* m) {
  if (!e || !m || rid_src >= e->nrep) return fail(RG_EINVAL, "rg_deliver args");
  const uint32_t R = e->c.replicas, K = e->c.max_msgs_per_pair, E = e->c.max_entries_per_msg;
  const uint64_t L = e->c.log_capacity;
  if (m->to < 1 || m->to > R) return fail(RG_EINVAL, "rg_deliver: bad destination");
  const uint32_t dst = m->to - 1;
  const int ob = (int)((e->t + 1) & 1);
  HIPCHK(hipStreamSynchronize(e->stream));
  uint32_t n = 0;
  uint32_t* cp = e->cnt[ob] + (uint64_t)rid_src * R + dst;
  HIPCHK(hipMemcpy(&n, cp, 4, hipMemcpyDeviceToHost));
  if (n >= K) return fail(RG_EFULL, "rg_deliver: outbox slot full");
  rg_msg_view h = *m;
  if (h.from == 0) h.from = (uint8_t)(rid_src % R + 1);
  if (h.type == RG_MSG_REPLICATE && h.nent) {
    if (h.nent > E) return fail(RG_EINVAL, "rg_deliver: too many entries");
    rg_replica_view v;
    int rc = rg_read_replicas(e, rid_src, 1, &v);
    if (rc) return rc;
    if (h.log_index < v.marker || h.log_index + h.nent > v.last) return fail(RG_EINVAL, "rg_deliver: entries not in sender log");
    std::vector<uint64_t> tv(h.nent);
    for (uint32_t k = 0; k < h.nent; ++k) {
      uint64_t slot = (h.log_index + 1 + k) & (L - 1);
      HIPCHK(hipMemcpy(&tv[k], e->term_ring + (uint64_t)rid_src * L + slot, 8, hipMemcpyDeviceToHost));
    }
    HIPCHK(hipMemcpy(e->mt[ob] + (((uint64_t)rid_src * R + dst) * K + n) * E, tv.data(), h.nent * 8ull,
                     hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemcpy(e->hdr[ob] + ((uint64_t)rid_src * R + dst) * K + n, &h, sizeof h, hipMemcpyHostToDevice));
  n++;
  HIPCHK(hipMemcpy(cp, &n, 4, hipMemcpyHostToDevice));
  return RG_OK;
}

int rg_leader(rg_engine* e, uint32_t group, uint64_t* leader_id, uint64_t* term, int* valid) {
  if (!e || group >= e->c.groups) return fail(RG_EINVAL, "rg_leader: bad group");
  std::vector<rg_replica_view> v(e->c.replicas);
  int rc = rg_read_replicas(e, group * e->c.replicas, e->c.replicas, v.data());
  if (rc) return rc;
  uint64_t bl = 0, bt = 0;
  for (auto& r : v) {
    if (r.term > bt) bt = r.term;
    if (r.role == RG_LEADER && r.term >= bt) bl = r.leader;
  }
  // the leader is valid only if it holds the highest term seen in the group
  uint64_t lt = 0;
  for (auto& r : v)
    if (r.role == RG_LEADER && r.leader == bl) lt = r.term;
  if (leader_id) *leader_id = (lt == bt) ? bl : 0;
  if (term) *term = bt;
  if (valid) *valid = (bl != 0 && lt == bt) ? 1 : 0;
  return RG_OK;
}

int rg_sum_committed(rg_engine* e, uint64_t* out) {
  if (!e || !out) return fail(RG_EINVAL, "rg_sum_committed args");
  HIPCHK(hipMemsetAsync(e->d_sum, 0, 8, e->stream));
  HIPCHK(launch_sum_committed(e->st[e->t & 1], e->c.groups, e->c.replicas, e->d_sum, e->stream));
  unsigned long long v = 0;
  HIPCHK(hipMemcpyAsync(&v, e->d_sum, 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  *out = v;
  return RG_OK;
}

int rg_last_tick_traffic(rg_engine* e, rg_traffic* out) {
  if (!e || !out) return fail(RG_EINVAL, "rg_last_tick_traffic args");
  if (e->t == 0) return fail(RG_EINVAL, "no tick has run");
  // the last tick read st[(t+1)&1] and wrote st[t&1], cnt/hdr[(t+1)&1] ... viewed as a tick input:
  TickParams p = params(e);  // p.st_in = current state, p.cnt_in/hdr_in = last tick's outbox
  HIPCHK(hipMemsetAsync(e->d_sum, 0, 64, e->stream));
  HIPCHK(launch_traffic(p, e->st[(e->t + 1) & 1], e->d_sum, e->stream));
  unsigned long long v[8] = {0};
  HIPCHK(hipMemcpyAsync(v, e->d_sum, 64, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  const uint64_t P = e->c.payload_bytes, R = e->c.replicas;
  out->replicas = e->nrep;
  out->leaders = v[0];
  out->msgs = v[1];
  out->repl_entries = v[2];
  out->appended = v[3];
  out->leader_appended = v[4];
  out->algorithmic_bytes = 128ull * e->nrep + 36ull * R * v[0] + 128ull * v[1] + (16 + P) * v[2] +
                           (12 + P) * v[3] + P * v[4];
  return RG_OK;
}

}  // extern "C"
