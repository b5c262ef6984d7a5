// raftgpu_engine.cpp — host runtime behind the C-ABI in include/raftgpu.h.
//
// Owns the device-resident structure-of-arrays replica table, builds the CRC
// tables, and issues each tick as two launches on the engine's stream: control_kernel<R>
// (Raft logic, one lane per replica) then bulk_kernel (payload + CRC). The product path has no
// CPU fallback: an engine cannot be created without a GPU and every rg_tick runs the kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <thread>
#include <unordered_map>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/raftgpu.h"
#include "raftgpu_internal.h"
#include "raftgpu_sdma.h"
#include "raftgpu_wire.h"

using namespace rg;

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                               \
  do {                                                                                          \
    hipError_t _e = (x);                                                                        \
    if (_e != hipSuccess) return fail(RG_EHIP, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

// Knobs (r05): the product reads no tuning knob from the environment. The A/B settings of earlier
// rounds are build-time variants for scripts/build_variant.sh (-DRG_AB_*); only four test hooks are
// read, once, at rg_create / rg_rccl_open: RAFTGPU_WIRE_CAP0 (start the fixed-capacity regions small),
// RAFTGPU_CTL_FB (force the control fallback in or out of the fast kernel's launch), RAFTGPU_APPLY_SDMA
// (the copy-back's D2H leg on an SDMA engine) and RAFTGPU_RCCL_SELF (rg_wire_exchange hands the region
// to self to the transport, which moves it through RCCL, instead of packing it in place) — each
// selects between two product paths the tests run bit-exact.
// RG_SYNC_DEBUG builds synchronise after every launch so a fault names its kernel (debug only).
#ifdef RG_SYNC_DEBUG
static constexpr bool g_sync_debug = true;
#else
static constexpr bool g_sync_debug = false;
#endif
#define LAUNCH(x, st, name)                                                                          \
  do {                                                                                              \
    HIPCHK(x);                                                                                      \
    if (g_sync_debug) {                                                                             \
      hipError_t _s = hipStreamSynchronize(st);                                                     \
      if (_s != hipSuccess) return fail(RG_EHIP, std::string(name) + ": " + hipGetErrorString(_s)); \
    }                                                                                               \
  } while (0)

#define RGCHK(x)             \
  do {                       \
    if (int _rc = (x)) return _rc; \
  } while (0)

constexpr uint32_t TP_SLOTS = 128, TP_CHUNK = 32;
constexpr uint32_t D_SUM_BYTES = 128;
static_assert(RG_RQ == RG_READ_QUEUE, "the ReadIndex queue rows and the ABI constant agree");  // rg_get_update's section totals (9 u64), digests, counters

// rg_propose's per-batch scratch (kept across calls)
struct PropScratch {
  std::vector<uint64_t> ch, by, mk, src, c0;  // chunks, payload bytes, non-empty mask, payload offset, arena chunk
  std::vector<uint32_t> nc0;                  // chunk count of the first Cmd
  std::vector<uint8_t> fl;                    // 1 uniform chunk count, 2 flat, 4 last Cmd a multiple of 16 B
  void resize(size_t n) {
    for (auto* v : {&ch, &by, &mk, &src, &c0}) v->resize(n);
    nc0.resize(n);
    fl.resize(n);
  }
};

// f(lo, hi) over [0, n) on T threads (the calling one included)
template <class F>
static void par_for(uint64_t T, uint64_t n, F&& f) {
  if (T <= 1 || n < 2) {
    f((size_t)0, (size_t)n);
    return;
  }
  std::vector<std::thread> th;
  for (uint64_t t = 1; t < T; ++t) th.emplace_back([&, t] { f((size_t)(n * t / T), (size_t)(n * (t + 1) / T)); });
  f((size_t)0, (size_t)(n / T));
  for (auto& x : th) x.join();
}

struct rg_engine {
  rg_config c{};
  uint32_t nrep = 0, J = 0;
  hipStream_t own = nullptr, stream = nullptr, bulk = nullptr;
  hipEvent_t ctl_done[2] = {nullptr, nullptr}, bulk_done[2] = {nullptr, nullptr};
  // replica state, updated in place by each step (a step writes only the fields it changes)
  uint64_t* s64 = nullptr;
  uint32_t* s32 = nullptr;
  uint64_t* rem = nullptr;
  uint8_t* rst = nullptr;
  uint64_t* tr = nullptr;
  uint2* info = nullptr;
  // paged payload streams: pool pages, per-replica page tables, the free-id ring and
  // its counters
  uint8_t* pool = nullptr;
  uint32_t* pt = nullptr;
  uint32_t* fring = nullptr;
  PoolCtl* poolctl = nullptr;
  uint64_t npages = 0;
  uint32_t PTS = 0, maxc = 0;  // stream pages per replica, longest Cmd
  uint64_t* hdr[2] = {nullptr, nullptr};
  uint64_t* mt[2] = {nullptr, nullptr};
  uint32_t* cnt[2] = {nullptr, nullptr};
  uint64_t* job64[2] = {nullptr, nullptr};  // double-buffered: control(t+1) overlaps bulk(t)
  uint32_t* job32[2] = {nullptr, nullptr};
  uint32_t* jcnt[2] = {nullptr, nullptr};
  uint32_t* crc_err = nullptr;
  uint8_t* slabs = nullptr;
  uint2* slab_info = nullptr;  // [nslab][rows][E] {SYN_OFF or arena chunk, Cmd length}
  // caller Cmds (rg_propose): one arena per slab, [nslab][cmd_cap], filled chunk-aligned from
  // cmd_used[slab] on by the H2D copy of a call; a slab's arena restarts when a new tick takes it
  uint8_t* cmds = nullptr;
  uint64_t cmd_cap = 0;
  std::vector<uint64_t> cmd_used, cmd_tick;
  uint64_t slab_synth = 0;  // bit s: slab s holds the generator's bytes (rg_fill_slabs, no rg_propose into it since)
  // caller proposals staged for the next tick (rg_propose): pinned host tables indexed by global input
  // index, uploaded by the tick; Cmd bytes + per-entry descriptors staged through pinned buffers
  uint8_t* h_pt = nullptr;
  uint32_t* h_pc = nullptr;
  uint64_t* h_hm = nullptr;
  uint64_t* d_prop_hmask = nullptr;
  // per shard: {stream chunks | contiguous in the arena << 31, arena chunk of entry 0} (pinned), and
  // the chunk count of its first Cmd (host only: a batch is contiguous while every Cmd has it)
  uint2* h_pcmd = nullptr;
  uint2* d_prop_cmd = nullptr;
  std::vector<uint32_t> pnc;
  // rg_propose scratch, kept across calls: per input index this call's additions (validation),
  // the indices set, the callers' Cmd offsets, and per staged Cmd its source offset
  std::vector<uint32_t> padd;
  std::vector<uint64_t> pset, pboff;
  PropScratch ps;                 // per batch of a call (rg_propose)
  std::vector<size_t> ppiece;     // first batch of each staged piece
  std::vector<std::pair<uintptr_t, uint64_t>> hreg;  // host ranges registered by rg_host_register
  std::vector<uint64_t> touched;  // input indices set in h_* since the last upload
  bool staged = false, stg_reset_pending = false;
  hipEvent_t stg_ev = nullptr;    // the last upload of h_* (host may rewrite them once it completed)
  hipEvent_t prop_ev = nullptr;   // the last H2D out of the pinned Cmd staging below
  uint8_t* h_cmd = nullptr;       // pinned: Cmd bytes, then off / dst (u64) and len (u32) per entry
  uint64_t h_cmd_cap = 0;
  uint8_t* d_cmd = nullptr;
  uint64_t d_cmd_cap = 0;
  // ReadIndex: device state rows, and the requests staged for the next tick (pinned table indexed
  // by global replica id, uploaded by the tick like the proposal tables)
  uint64_t* rdst = nullptr;
  uint64_t* h_rd = nullptr;
  uint64_t* d_read_ctx = nullptr;
  std::vector<uint64_t> rd_touched;
  bool rd_staged = false, rd_reset_pending = false;
  hipEvent_t rd_ev = nullptr;
  // rg_config_change staging: [global group] slot | descriptor << 8 (pinned), uploaded by the tick
  uint16_t* h_cc = nullptr;
  uint16_t* d_cc = nullptr;
  std::vector<uint64_t> cc_touched;
  bool cc_staged = false, cc_reset_pending = false;
  hipEvent_t cc_ev = nullptr;
  uint32_t* crc_tab = nullptr;
  uint32_t crc_const = 0;
  uint8_t* d_prop_target = nullptr;
  uint32_t* d_prop_count = nullptr;
  uint8_t* d_campaign = nullptr;
  uint8_t* d_isolate = nullptr;
  unsigned long long* d_sum = nullptr;  // D_SUM_BYTES: small totals read back by the host
  // control_kernel's parameter block, passed by pointer (DESIGN.md §3 "The control-kernel fault"):
  // TP_SLOTS device slots, written by stream-ordered H2D copies from pinned host slots of the same
  // index: at a chunk's first tick one copy of the whole chunk, whose blocks are speculated for the
  // next TP_CHUNK ticks with that tick's inputs (h_tp); a later tick of the chunk whose block differs
  // copies its own (h_fb). tp_ev[c] follows chunk c's last launch, so a host slot is rewritten only
  // after the copies out of it (TP_SLOTS launches earlier) have completed
  TickParams* d_tp = nullptr;
  TickParams* h_tp = nullptr;
  TickParams* h_fb = nullptr;
  uint64_t tp_copies = 0;  // parameter-block copies issued (rg_debug_param_copies)
  hipEvent_t tp_ev[TP_SLOTS / TP_CHUNK] = {};
  bool tp_used[TP_SLOTS / TP_CHUNK] = {};
  uint64_t tp_next = 0;
  uint32_t tp_corrupt = 0;  // tests (rg_debug_corrupt_params): seal the next n blocks with a wrong checksum
  // the control fast path: control_fast_kernel then control_slow_kernel over the replicas it
  // handed off ([2] counters by tick parity, then the list); build variant -DRG_AB_CTL_FULL: control_kernel alone
  uint32_t* slow = nullptr;
  bool ctl_fast = true;
  bool ctl_fb = false;  // small engines: the fallback runs in the fast kernel's launch (control_fastfb_kernel)
  uint8_t* stage = nullptr;
  uint64_t stage_bytes = 0;
  uint64_t t = 0;
  int bulk_grid = 0;
  uint32_t bulk_tile = 1;
  // small jobs share a bulk ring pass (bulk_kernel<.., MJ = true>): when Replicates and proposal
  // batches carry at most 16 entries (max_entries_per_msg), jobs are small; the 64-entry jobs of
  // full batches run faster without it. Build variant -DRG_AB_BULK_MULTIJOB=0/1 overrides.
  bool bulk_mj = false;
  bool bulk_small = true;
  uint32_t bulk_wg = 4;  // waves per bulk workgroup; MJ engines: bulk_small_kernel takes the small jobs first (-DRG_AB_NO_BULK_SMALL: off)
  uint64_t bytes = 0;
  std::vector<void*> allocs;
  // per-launch event timing (rg_timing): bit 0 control_kernel, bit 1 bulk_kernel; a start/end
  // event pair per timed launch
  int timing = 0;
  uint32_t timing_every = 1;
  std::vector<hipEvent_t> ev_pool, ev_live;
  std::vector<int> ev_kind;  // kernel (0 control, 1 bulk) of each start/end pair in ev_live
  std::vector<uint64_t> ev_tick;  // the tick of each pair
  struct KEvent { uint64_t tick; double start, end; };
  std::vector<KEvent> kev[2];  // timed launches on the process epoch's timeline (rg_timing_epoch)
  double kms[2] = {0, 0};
  uint64_t klaunch[2] = {0, 0};
  uint32_t T0[256];
  // placement + inter-rank exchange
  Placement pl{};
  bool wire = false;            // some plane crosses ranks (ranks > 1 or wire_all)
  uint32_t slab_rows = 0;
  uint32_t *umap = nullptr, *ubeg = nullptr, *rmap = nullptr, *rbeg = nullptr;
  uint32_t U = 0, RU = 0;
  std::vector<uint32_t> h_ubeg, h_rbeg;
  uint32_t* usize = nullptr;
  uint64_t *uoff = nullptr, *bsum = nullptr, *bounds = nullptr, *h_bounds = nullptr;
  uint64_t* rhdr = nullptr;
  uint64_t* rmt = nullptr;
  uint32_t* rcnt = nullptr;
  std::vector<uint64_t> send_bytes;
  bool planned = false, wire_ready = false;
  // fixed-capacity exchange (rg_wire_plan_fixed): region bytes per peer, the same at
  // both ends of a link (the same rule over the same numbers), grown from the exchange two before
  std::vector<uint64_t> cap_s, cap_r, cap_s0, cap_r0;  // capacities now, and their floors
  std::vector<uint64_t> win_s, win_r;  // [N][WIRE_WIN] needs of the last exchanges, per link
  uint64_t* d_need = nullptr;  // [2][MAX_RANKS]: bytes each sent region asked for (pack), each received one (unpack)
  uint64_t* h_need = nullptr;  // pinned [4][2][MAX_RANKS], one slot per exchange
  hipEvent_t need_ev[4] = {nullptr, nullptr, nullptr, nullptr};
  uint64_t nfix = 0;           // fixed-capacity exchanges so far
  bool fixed = false;          // the planned exchange is fixed-capacity
  unsigned long long* d_drops = nullptr;  // messages dropped by a full region (cumulative)
  const uint8_t* recv = nullptr;  // receive buffer the next tick's SRC_WIRE jobs read
  uint64_t recv_bytes = 0;         // bytes of it in use (RG_BOUNDS checks)
  // rg_wire_exchange's own buffers (grown on demand; stream order keeps one of each enough: the
  // next exchange is enqueued after the tick that reads the receive buffer)
  uint8_t* x_recv = nullptr;  // rg_wire_exchange's buffer: receive regions, then send regions
  uint64_t x_recv_cap = 0;
  bool self_via_transport = false;  // RAFTGPU_RCCL_SELF=rccl (tests): no in-place region to self
  // committed-entry copy-back (raftgpu_apply.hip)
  uint64_t* feed = nullptr;  // [nrep] the last tick's hand-off words (feed_word: apply window, persist, snapshots)
  uint32_t* small_rest = nullptr;  // BulkParams::rest
  uint64_t* rest_tick = nullptr;   // BulkParams::rest_tick
  uint32_t *acnt = nullptr, *accnt = nullptr, *arcnt = nullptr;
  uint64_t *aoff = nullptr, *acoff = nullptr, *aroff = nullptr, *absum = nullptr;
  bool copy_kernel = true;  // build variant -DRG_AB_APPLY_MEMCPY: the runtime's D2H copy instead
  SdmaCopier* sdma = nullptr;  // RAFTGPU_APPLY_SDMA=1: the D2H leg on an SDMA engine (raftgpu_sdma.cpp)
  uint8_t* astage = nullptr;
  uint64_t astage_bytes = 0;
  // asynchronous copy-back (rg_apply_async): per buffer a device staging area, pinned host memory,
  // and events for "gathered" and "copied"; copies run on their own stream
  hipStream_t copy = nullptr;
  hipEvent_t a_gath[2] = {nullptr, nullptr}, a_copy[2] = {nullptr, nullptr};
  uint8_t* a_dev[2] = {nullptr, nullptr};
  uint8_t* ac_host = nullptr;  // rg_apply_committed's pinned batch
  uint64_t ac_hcap = 0;
  uint64_t a_tot[2][3] = {};   // rg_apply_async: the batch's entries, chunks, runs per buffer
  uint8_t* a_host[2] = {nullptr, nullptr};
  uint64_t a_dcap[2] = {0, 0}, a_hcap[2] = {0, 0}, a_n[2] = {0, 0};
  bool a_used[2] = {false, false};
  // persistence copy-back
  uint32_t* prof = nullptr;     // RG_CTL_PROFILE builds: control phase stamps of the last tick
  uint32_t *pscnt = nullptr, *pecnt = nullptr, *pccnt = nullptr, *ptcnt = nullptr;
  uint64_t *psoff = nullptr, *peoff = nullptr, *pcoff = nullptr, *ptoff = nullptr;
  uint8_t* pc_host = nullptr;  // rg_persist_collect's pinned batch
  uint64_t pc_hcap = 0;
  // rg_get_update: count / offset rows of the snapshot and read sections (the committed section
  // uses acnt / aoff, the persistence section pscnt / psoff, so every count runs before any gather),
  // and the pinned host buffer all sections land in
  uint32_t *uscnt = nullptr, *urcnt = nullptr;
  uint64_t *usoff = nullptr, *uroff = nullptr;
  uint8_t* u_host = nullptr;
  uint64_t u_hcap = 0;
  // rg_tick_device_n's HIP graphs ("Multi-tick path"): two captured graphs of g_k ticks,
  // each over its own set of parameter slots, used alternately so the host refills one set while
  // the other graph may still be reading its slots; g_ev[i] follows the last launch of graph i
  hipGraph_t gg[2] = {nullptr, nullptr};
  hipGraphExec_t gx[2] = {nullptr, nullptr};
  hipEvent_t g_ev[2] = {nullptr, nullptr};
  bool g_used[2] = {false, false}, g_valid = false;
  uint32_t g_k = 0, g_par = 0, g_flip = 0;
  rg_tick_input g_in{};
  hipStream_t g_stream = nullptr;
  TickParams* g_dtp = nullptr;  // [2][G_MAXK] device slots
  TickParams* g_htp = nullptr;  // [2][G_MAXK] pinned host slots
};
constexpr uint32_t G_MAXK = 64;

static int stage_reset(rg_engine* e);

// ---------------------------------------------------------------- CRC-32 tables
// Reflected CRC-32, init and xorout 0xFFFFFFFF: IEEE (zlib) or Castagnoli (rg_config.crc32c).
// Everything the kernels use (byte, nibble and shift tables, the finalisation constant) is built
// here, so the device code is the same for both polynomials.
static void build_crc(rg_engine* e, std::vector<uint32_t>& tab) {
  uint32_t* T0 = e->T0;
  const uint32_t poly = e->c.crc32c ? 0x82F63B78u : 0xEDB88320u;
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : c >> 1;
    T0[b] = c;
  }
  auto Z = [&](uint32_t x) { return T0[x & 0xFF] ^ (x >> 8); };  // one zero byte
  auto Zn = [&](uint32_t x, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) x = Z(x);
    return x;
  };
  tab.assign(CRC_TAB_WORDS, 0);
  for (uint32_t k = 0; k < 16; ++k)
    for (uint32_t b = 0; b < 256; ++b) tab[k * 256 + b] = Zn(T0[b], k);
  for (uint32_t k = 0; k < 16; ++k)
    for (uint32_t n = 0; n < 16; ++n) {
      tab[CRC_T_WORDS + (k * 2 + 0) * 16 + n] = tab[k * 256 + n];
      tab[CRC_T_WORDS + (k * 2 + 1) * 16 + n] = tab[k * 256 + (n << 4)];
    }
  const uint32_t nch = e->c.payload_bytes / 16;
  for (uint32_t c = 0; c < nch; ++c)
    for (uint32_t j = 0; j < 8; ++j)
      for (uint32_t n = 0; n < 16; ++n)
        tab[CRC_T_WORDS + CRC_N_WORDS + c * CRC_SH_STRIDE + j * 16 + n] = Zn(n << (4 * j), 16 * (nch - 1 - c));
  e->crc_const = Zn(0xFFFFFFFFu, e->c.payload_bytes) ^ 0xFFFFFFFFu;
  // inverse shifts: Z(x) = T0[x & 0xFF] ^ (x >> 8) is invertible (the top byte of T0[b] names b)
  uint32_t top[256];
  for (uint32_t b = 0; b < 256; ++b) top[T0[b] >> 24] = b;
  auto Zi = [&](uint32_t y) {
    const uint32_t b = top[y >> 24];
    return ((y ^ T0[b]) << 8) | b;
  };
  for (uint32_t b = 0; b < CRC_ZI_BITS; ++b)
    for (uint32_t j = 0; j < 8; ++j)
      for (uint32_t n = 0; n < 16; ++n) {
        uint32_t x = n << (4 * j);
        for (uint32_t i = 0; i < (1u << b); ++i) x = Zi(x);
        tab[CRC_ZI_OFF + (b * 8 + j) * 16 + n] = x;
      }
  // Z^P (chaining the P-byte segments of a longer Cmd)
  const uint32_t P = e->c.payload_bytes;
  for (uint32_t j = 0; j < 8; ++j)
    for (uint32_t n = 0; n < 16; ++n) tab[CRC_ZP_OFF + j * 16 + n] = Zn(n << (4 * j), P);
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
  if (r != hipSuccess) return fail(RG_ENOMEM, "hipMalloc(" + std::to_string(bytes) + " B) failed: " + hipGetErrorString(r));
  e->allocs.push_back(*p);
  e->bytes += bytes;
  return RG_OK;
}

static int stage_reserve(rg_engine* e, uint64_t bytes) {
  if (bytes <= e->stage_bytes) return RG_OK;
  if (e->stage) {
    (void)hipStreamSynchronize(e->stream);
    (void)hipFree(e->stage);
    e->allocs.erase(std::remove(e->allocs.begin(), e->allocs.end(), (void*)e->stage), e->allocs.end());
    e->bytes -= e->stage_bytes;
    e->stage = nullptr;
    e->stage_bytes = 0;
  }
  const uint64_t nb = std::max<uint64_t>(bytes, 1 << 20);
  int rc = dalloc(e, &e->stage, nb);
  if (rc == RG_OK) e->stage_bytes = nb;
  return rc;
}

static bool pow2(uint32_t x) { return x && !(x & (x - 1)); }
static uint64_t a16(uint64_t x) { return (x + 15) & ~15ull; }

// The parameter block of the tick that runs next (tick e->t): reads parity t&1 state and the
// outbox written by tick t-1, writes the other parity.
static TickParams params_at(rg_engine* e, uint64_t t);
static TickParams params(rg_engine* e) { return params_at(e, e->t); }
static TickParams params_at(rg_engine* e, uint64_t tk) {
  TickParams p{};
  const rg_config& c = e->c;
  p.G = c.groups; p.R = c.replicas; p.nrep = e->nrep; p.L = c.log_capacity; p.P = c.payload_bytes;
  p.E = c.max_entries_per_msg; p.K = c.max_msgs_per_pair; p.nslab = c.num_slabs; p.J = e->J;
  p.ET = c.election_rtt; p.HT = c.heartbeat_rtt; p.CQ = c.check_quorum; p.SE = c.snapshot_entries;
  p.CO = c.compaction_overhead; p.drop_ppm = c.drop_ppm;
  p.wire = e->wire ? 1u : 0u;
  p.AF = c.apply_feedback;
  p.PTS = e->PTS;
  p.JS = c.join_slots;
  p.IM = c.initial_members;
  p.seed = c.seed;
  p.tick = tk;
  p.pl = e->pl;
  const int a = (int)(tk & 1), b = a ^ 1;
  p.s64 = e->s64; p.s32 = e->s32; p.rem = e->rem; p.rst = e->rst;
  p.tr = e->tr;
  p.hdr_in = e->hdr[b]; p.hdr_out = e->hdr[a];
  p.mt_in = e->mt[b]; p.mt_out = e->mt[a];
  p.cnt_in = e->cnt[b]; p.cnt_out = e->cnt[a];
  p.job64 = e->job64[a]; p.job32 = e->job32[a]; p.jcnt = e->jcnt[a];
  p.rhdr = e->rhdr; p.rmt = e->rmt; p.rcnt = e->rcnt;
  p.slab_info = e->slab_info;
  p.rdst = e->rdst;
  p.feed = e->feed;
  p.prof = e->prof;
  p.info = e->info;
  p.pool = e->poolctl;
  if (e->ctl_fast) {
    p.slow_cnt = e->slow;
    p.slow_flag = e->slow + 2;
  }
  return p;
}

static WireParams wire_params(rg_engine* e) {
  const TickParams p = params(e);
  WireParams w{};
  w.G = p.G; w.R = p.R; w.nrep = p.nrep; w.L = p.L; w.P = p.P; w.E = p.E; w.K = p.K;
  w.pl = e->pl;
  w.hdr = p.hdr_in; w.mt = p.mt_in; w.cnt = p.cnt_in;
  w.info = e->info; w.pool = e->pool; w.pt = e->pt; w.PTS = e->PTS; w.maxc = e->maxc;
  w.slabs = e->slabs; w.slab_info = e->slab_info; w.nslab = e->c.num_slabs;
  w.cmds = e->cmds; w.cmd_cap = e->cmd_cap;
  w.umap = e->umap; w.ubeg = e->ubeg; w.U = e->U;
  w.usize = e->usize; w.uoff = e->uoff; w.bsum = e->bsum;
  w.rmap = e->rmap; w.rbeg = e->rbeg; w.RU = e->RU;
  w.rhdr = e->rhdr; w.rmt = e->rmt; w.rcnt = e->rcnt;
  w.sneed = e->d_need; w.rneed = e->d_need ? e->d_need + MAX_RANKS : nullptr; w.drops = e->d_drops;
  return w;
}

static BulkParams bulk_params_at(rg_engine* e, uint64_t tk);
static BulkParams bulk_params(rg_engine* e) { return bulk_params_at(e, e->t); }
static BulkParams bulk_params_at(rg_engine* e, uint64_t tk) {
  const int a = (int)(tk & 1);
  BulkParams b{};
  b.G = e->c.groups; b.R = e->c.replicas; b.nrep = e->nrep; b.L = e->c.log_capacity; b.P = e->c.payload_bytes;
  b.E = e->c.max_entries_per_msg; b.J = e->J; b.crc_const = e->crc_const; b.tile = e->bulk_tile;
  b.job64 = e->job64[a]; b.job32 = e->job32[a]; b.jcnt = e->jcnt[a];
  b.tr = e->tr; b.info = e->info; b.pool = e->pool; b.PTS = e->PTS;
  b.slabs = e->slabs; b.slab_info = e->slab_info; b.cmds = e->cmds; b.cmd_cap = e->cmd_cap;
  b.crc_err = e->crc_err; b.crc_tab = e->crc_tab; b.poolctl = e->poolctl;
  b.wire_mode = e->wire ? 1u : 0u;
  b.wire = e->recv;
  b.wire_bytes = e->recv_bytes;
  b.nslab = e->c.num_slabs;
  b.multijob = e->bulk_mj ? 1u : 0u;
  b.small = e->bulk_mj && e->bulk_small ? 1u : 0u;
  b.rest = e->small_rest;
  b.rest_tick = e->rest_tick;
  b.tick = tk;
  b.wg_waves = e->bulk_wg;
  return b;
}

static AdminParams admin(rg_engine* e) {
  AdminParams a{};
  a.t = params(e);
  a.info = e->info;
  a.pool = e->pool;
  a.pt = e->pt;
  a.PTS = e->PTS;
  a.row = e->maxc;
  a.fring = e->fring;
  a.npages = e->npages;
  a.poolctl = e->poolctl;
  a.crc_err = e->crc_err;
  a.zi = e->crc_tab + CRC_ZI_OFF;
  return a;
}

extern "C" {

const char* rg_last_error(void) { return g_err.c_str(); }

int rg_create(const rg_config* cfg, rg_engine** out) {
  if (!cfg || !out) return fail(RG_EINVAL, "null argument");
  const rg_config& c = *cfg;
  if (c.groups < 1 || c.replicas < 1 || c.replicas > RG_MAX_REPLICAS) return fail(RG_EINVAL, "groups/replicas");
  if (!pow2(c.log_capacity) || c.log_capacity < 16 || c.log_capacity > (1u << 28))
    return fail(RG_EINVAL, "log_capacity must be a power of two in [16, 2^28]");
  if (c.payload_bytes && (!pow2(c.payload_bytes) || c.payload_bytes < 16 || c.payload_bytes > 1024))
    return fail(RG_EINVAL, "payload_bytes must be 0 or a power of two in [16, 1024]");
  if (c.max_entries_per_msg < 1 || c.max_entries_per_msg > 64) return fail(RG_EINVAL, "max_entries_per_msg in 1..64");
  if (c.max_msgs_per_pair < 1 || c.max_msgs_per_pair > 16) return fail(RG_EINVAL, "max_msgs_per_pair in 1..16");
  if (c.num_slabs < 2 || c.num_slabs > 64 || c.election_rtt < 1 || c.heartbeat_rtt < 1)
    return fail(RG_EINVAL, "num_slabs in 2..64, rtt >= 1");
  if ((uint64_t)c.groups * c.replicas > 0x7FFFFFFFull) return fail(RG_EINVAL, "too many replicas");
  const uint32_t N = c.ranks ? c.ranks : 1;
  if (N > MAX_RANKS || c.rank >= N) return fail(RG_EINVAL, "ranks in 1..16, rank < ranks");
  if (c.crc32c > 1) return fail(RG_EINVAL, "crc32c must be 0 (IEEE) or 1 (Castagnoli)");
  if (c.apply_feedback > 1) return fail(RG_EINVAL, "apply_feedback must be 0 or 1");
  if (c.initial_members >> c.replicas) return fail(RG_EINVAL, "initial_members names a slot >= replicas");
  if ((N > 1 || c.wire_all) && c.groups >= (1u << 24)) return fail(RG_EINVAL, "groups < 2^24 with ranks > 1");
  const uint32_t maxc = c.max_cmd_bytes ? c.max_cmd_bytes : c.payload_bytes;
  if (c.payload_bytes ? (maxc < c.payload_bytes || maxc > MAX_CMD) : maxc != 0)
    return fail(RG_EINVAL, "max_cmd_bytes must be in [payload_bytes, 16 MiB] (0 with payload_bytes 0)");
  if (c.stream_pages && (!pow2(c.stream_pages) || c.stream_pages > (1u << 20)))
    return fail(RG_EINVAL, "stream_pages must be 0 or a power of two <= 2^20");
  if (c.pool_pages > (1u << 24)) return fail(RG_EINVAL, "pool_pages <= 2^24 (64 GiB)");
  if (c.join_slots >> c.replicas) return fail(RG_EINVAL, "join_slots names a slot >= replicas");
  if (c.initial_members & c.join_slots) return fail(RG_EINVAL, "a slot is both an initial member and joining");
  if (c.join_slots == (1u << c.replicas) - 1u) return fail(RG_EINVAL, "every slot joining: nobody to join");
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (ndev <= 0 || c.device < 0 || c.device >= ndev) return fail(RG_EINVAL, "no such HIP device");
  HIPCHK(hipSetDevice(c.device));

  rg_engine* e = new rg_engine();
  e->c = c;
  e->c.ranks = N;
  e->nrep = c.groups * c.replicas;
  e->pl = make_placement(N, c.rank, c.wire_all, c.column_base);
  e->wire = N > 1 || c.wire_all;
  e->slab_rows = e->wire ? e->nrep : c.groups;  // wire engines: one slab row per replica (bulk_kernel<LG, true>)
  e->J = (c.replicas - 1) * c.max_msgs_per_pair + 2;  // >= appends one step can make
  e->maxc = maxc;
  {  // payload streams: a replica's window (auto: twice a full log of P-byte Cmds, plus room for two of
     // the longest Cmds when max_cmd_bytes > P; oracle.c sizes it the same way) and the pool
    const uint64_t full = ((uint64_t)c.log_capacity * ((c.payload_bytes + 15) & ~15u) + PAGE_BYTES - 1) / PAGE_BYTES;
    const uint64_t big = maxc > c.payload_bytes ? 2 * ((maxc + PAGE_BYTES - 1) / PAGE_BYTES + 1) : 0;
    uint32_t pts = 16;
    while (pts < 2 * full + big) pts <<= 1;
    e->PTS = c.payload_bytes ? (c.stream_pages ? c.stream_pages : pts) : 1;
    const uint64_t want = (uint64_t)c.groups * c.replicas * (full + 2);
    e->npages = !c.payload_bytes ? 0 : c.pool_pages ? c.pool_pages : std::min<uint64_t>(want, 1ull << 24);
  }
  const uint64_t n = e->nrep, L = c.log_capacity, P = c.payload_bytes, R = c.replicas, K = c.max_msgs_per_pair,
                 E = c.max_entries_per_msg, G = c.groups, J = e->J;
  int rc = RG_OK;
  rc = dalloc(e, &e->s64, S64_ROWS * n * 8);
  if (rc == RG_OK) rc = dalloc(e, &e->s32, S32_ROWS * n * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->rem, 3 * R * n * 8);
  if (rc == RG_OK) rc = dalloc(e, &e->rst, R * n);
  for (int b = 0; b < 2 && rc == RG_OK; ++b) {
    rc = dalloc(e, &e->hdr[b], 8 * R * R * K * G * 8);
    if (rc == RG_OK) rc = dalloc(e, &e->mt[b], R * R * K * E * G * 8);
    if (rc == RG_OK) rc = dalloc(e, &e->cnt[b], R * R * G * 4);
  }
  if (rc == RG_OK) rc = dalloc(e, &e->tr, L * n * 8);
  if (rc == RG_OK) rc = dalloc(e, &e->info, 2 * n * L * sizeof(uint2));
  if (rc == RG_OK) rc = dalloc(e, &e->pool, e->npages * PAGE_BYTES);
  if (rc == RG_OK) rc = dalloc(e, &e->pt, (uint64_t)n * e->PTS * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->fring, e->npages * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->poolctl, sizeof(PoolCtl));
  for (int b = 0; b < 2 && rc == RG_OK; ++b) {
    rc = dalloc(e, &e->job64[b], J64_ROWS * J * n * 8);
    if (rc == RG_OK) rc = dalloc(e, &e->job32[b], J32_ROWS * J * n * 4);
    if (rc == RG_OK) rc = dalloc(e, &e->jcnt[b], n * 4);
  }
  if (rc == RG_OK) rc = dalloc(e, &e->crc_err, n * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->slow, (n + 2) * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->slabs, (uint64_t)c.num_slabs * e->slab_rows * E * P);
  if (rc == RG_OK) rc = dalloc(e, &e->slab_info, (uint64_t)c.num_slabs * e->slab_rows * E * sizeof(uint2));
  e->cmd_used.assign(c.num_slabs, 0);
  e->cmd_tick.assign(c.num_slabs, ~0ull);
  if (rc == RG_OK) rc = dalloc(e, &e->d_prop_hmask, G * N * 8);
  if (rc == RG_OK) rc = dalloc(e, &e->d_prop_cmd, G * N * 8);
  if (rc == RG_OK && hipHostMalloc((void**)&e->h_pcmd, G * N * 8, 0) != hipSuccess)
    rc = fail(RG_ENOMEM, "hipHostMalloc (proposal tables)");
  if (rc == RG_OK) memset(e->h_pcmd, 0, G * N * 8);
  e->pnc.assign(G * N, 0);
  if (rc == RG_OK) rc = dalloc(e, &e->rdst, (uint64_t)RD_ROWS * n * 8);
  if (rc == RG_OK) rc = dalloc(e, &e->d_read_ctx, n * N * 8);
  if (rc == RG_OK && hipHostMalloc((void**)&e->h_rd, n * N * 8, 0) != hipSuccess) rc = fail(RG_ENOMEM, "hipHostMalloc");
  if (rc == RG_OK) memset(e->h_rd, 0, n * N * 8);
  if (rc == RG_OK) rc = dalloc(e, &e->d_cc, G * N * 2);
  if (rc == RG_OK && hipHostMalloc((void**)&e->h_cc, G * N * 2, 0) != hipSuccess) rc = fail(RG_ENOMEM, "hipHostMalloc");
  if (rc == RG_OK) memset(e->h_cc, 0, G * N * 2);
  if (rc == RG_OK && (hipHostMalloc((void**)&e->h_pt, G * N, 0) != hipSuccess ||
                      hipHostMalloc((void**)&e->h_pc, G * N * 4, 0) != hipSuccess ||
                      hipHostMalloc((void**)&e->h_hm, G * N * 8, 0) != hipSuccess))
    rc = fail(RG_ENOMEM, "hipHostMalloc (proposal tables)");
  if (rc == RG_OK) {
    memset(e->h_pt, 0xFF, G * N);
    memset(e->h_pc, 0, G * N * 4);
    memset(e->h_hm, 0, G * N * 8);
  }
  if (rc == RG_OK) rc = dalloc(e, &e->crc_tab, CRC_TAB_WORDS * 4);
  // tick inputs are indexed by global group / replica: ranks × the local sizes
  if (rc == RG_OK) rc = dalloc(e, &e->d_prop_target, G * N);
  if (rc == RG_OK) rc = dalloc(e, &e->d_prop_count, G * N * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->d_campaign, n * N);
  if (rc == RG_OK) rc = dalloc(e, &e->d_isolate, n * N);
  if (rc == RG_OK) rc = dalloc(e, &e->d_sum, D_SUM_BYTES);
  if (rc == RG_OK) rc = dalloc(e, &e->d_tp, (uint64_t)TP_SLOTS * sizeof(TickParams));
  if (rc == RG_OK && (hipHostMalloc((void**)&e->h_tp, (uint64_t)TP_SLOTS * sizeof(TickParams), 0) != hipSuccess ||
                      hipHostMalloc((void**)&e->h_fb, (uint64_t)TP_SLOTS * sizeof(TickParams), 0) != hipSuccess))
    rc = fail(RG_ENOMEM, "hipHostMalloc (parameter blocks)");
  if (rc == RG_OK) rc = dalloc(e, &e->feed, n * 8);
  if (rc == RG_OK) rc = dalloc(e, &e->acnt, n * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->accnt, n * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->aoff, (n + 1) * 8);
  if (rc == RG_OK) rc = dalloc(e, &e->acoff, (n + 1) * 8);
  if (rc == RG_OK) rc = dalloc(e, &e->arcnt, n * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->small_rest, (uint64_t)((c.groups + 63) / 64) * c.replicas * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->rest_tick, 8);
  if (rc == RG_OK && hipMemset(e->rest_tick, 0xFF, 8) != hipSuccess) rc = fail(RG_EHIP, "hipMemset (rest stamp)");
  if (rc == RG_OK) rc = dalloc(e, &e->aroff, (n + 1) * 8);
  if (rc == RG_OK) rc = dalloc(e, &e->absum, ((n + 1023) / 1024 + 1) * 8);
#ifdef RG_CTL_PROFILE
  if (rc == RG_OK) rc = dalloc(e, &e->prof, n * 12 * 4);
#endif
  if (rc == RG_OK) rc = dalloc(e, &e->pscnt, n * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->pecnt, n * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->pccnt, n * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->psoff, (n + 1) * 8);
  if (rc == RG_OK) rc = dalloc(e, &e->peoff, (n + 1) * 8);
  if (rc == RG_OK) rc = dalloc(e, &e->pcoff, (n + 1) * 8);
  if (rc == RG_OK) rc = dalloc(e, &e->ptcnt, n * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->ptoff, (n + 1) * 8);
  if (rc == RG_OK) rc = dalloc(e, &e->uscnt, n * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->urcnt, n * 4);
  if (rc == RG_OK) rc = dalloc(e, &e->usoff, (n + 1) * 8);
  if (rc == RG_OK) rc = dalloc(e, &e->uroff, (n + 1) * 8);
  // exchange units: every remote (s, d, j) outbox column, per destination rank (send) and per
  // source rank (receive), each in (s, d, j) order — the same list on both ends of a link
  if (rc == RG_OK && e->wire) {
    std::vector<std::vector<uint32_t>> snd(N), rcv(N);
    for (uint32_t s = 0; s < R; ++s)
      for (uint32_t d = 0; d < R; ++d) {
        if (s == d) continue;
        for (uint32_t j = 0; j < G; ++j) {
          if (!pl_remote(e->pl, s, d, j)) continue;
          const uint32_t off = pl_off(e->pl, s, d, j), code = (s << 28) | (d << 24) | j;
          snd[(c.rank + off) % N].push_back(code);
          rcv[(c.rank + N - off) % N].push_back(code);
        }
      }
    std::vector<uint32_t> um, rm;
    e->h_ubeg.assign(N + 1, 0);
    e->h_rbeg.assign(N + 1, 0);
    for (uint32_t r = 0; r < N; ++r) {
      e->h_ubeg[r] = (uint32_t)um.size();
      um.insert(um.end(), snd[r].begin(), snd[r].end());
      e->h_rbeg[r] = (uint32_t)rm.size();
      rm.insert(rm.end(), rcv[r].begin(), rcv[r].end());
    }
    e->h_ubeg[N] = (uint32_t)um.size();
    e->h_rbeg[N] = (uint32_t)rm.size();
    e->U = (uint32_t)um.size();
    e->RU = (uint32_t)rm.size();
    const uint64_t nb = (e->U + 1023) / 1024 + 1;
    rc = dalloc(e, &e->umap, (uint64_t)e->U * 4);
    if (rc == RG_OK) rc = dalloc(e, &e->rmap, (uint64_t)e->RU * 4);
    if (rc == RG_OK) rc = dalloc(e, &e->ubeg, (N + 1) * 4);
    if (rc == RG_OK) rc = dalloc(e, &e->rbeg, (N + 1) * 4);
    if (rc == RG_OK) rc = dalloc(e, &e->usize, (uint64_t)e->U * 4);
    if (rc == RG_OK) rc = dalloc(e, &e->uoff, ((uint64_t)e->U + 1) * 8);
    if (rc == RG_OK) rc = dalloc(e, &e->bsum, nb * 8);
    if (rc == RG_OK) rc = dalloc(e, &e->bounds, (MAX_RANKS + 1) * 8);
    if (rc == RG_OK) rc = dalloc(e, &e->rhdr, 8 * R * R * K * G * 8);
    if (rc == RG_OK) rc = dalloc(e, &e->rmt, R * R * K * E * G * 8);
    if (rc == RG_OK) rc = dalloc(e, &e->rcnt, R * R * G * 4);
    if (rc == RG_OK && hipHostMalloc((void**)&e->h_bounds, (MAX_RANKS + 1) * 8, 0) != hipSuccess)
      rc = fail(RG_ENOMEM, "hipHostMalloc");
    if (rc == RG_OK) rc = dalloc(e, &e->d_need, 2 * MAX_RANKS * 8);
    if (rc == RG_OK) rc = dalloc(e, &e->d_drops, 8);
    if (rc == RG_OK && hipHostMalloc((void**)&e->h_need, 4 * 2 * MAX_RANKS * 8, 0) != hipSuccess)
      rc = fail(RG_ENOMEM, "hipHostMalloc");
    for (int i = 0; i < 4 && rc == RG_OK; ++i)
      if (hipEventCreateWithFlags(&e->need_ev[i], hipEventDisableTiming) != hipSuccess) rc = fail(RG_EHIP, "event");
    if (rc == RG_OK && (hipMemset(e->d_need, 0, 2 * MAX_RANKS * 8) != hipSuccess ||
                        hipMemset(e->d_drops, 0, 8) != hipSuccess))
      rc = fail(RG_EHIP, "hipMemset");
    if (rc == RG_OK &&
        (hipMemcpy(e->umap, um.data(), um.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
         hipMemcpy(e->rmap, rm.data(), rm.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
         hipMemcpy(e->ubeg, e->h_ubeg.data(), (N + 1) * 4, hipMemcpyHostToDevice) != hipSuccess ||
         hipMemcpy(e->rbeg, e->h_rbeg.data(), (N + 1) * 4, hipMemcpyHostToDevice) != hipSuccess))
      rc = fail(RG_EHIP, "unit map upload");
    e->send_bytes.assign(N, 0);
  }
  if (rc != RG_OK) {
    std::string msg = g_err;
    rg_destroy(e);
    return fail(rc, msg);
  }
  if (hipStreamCreateWithFlags(&e->own, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&e->bulk, hipStreamNonBlocking) != hipSuccess) {
    rg_destroy(e);
    return fail(RG_EHIP, "hipStreamCreate");
  }
  for (int b = 0; b < 2; ++b) {
    if (hipEventCreateWithFlags(&e->ctl_done[b], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->bulk_done[b], hipEventDisableTiming) != hipSuccess) {
      rg_destroy(e);
      return fail(RG_EHIP, "hipEventCreate");
    }
  }
  if (hipEventCreateWithFlags(&e->rd_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->cc_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->stg_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->prop_ev, hipEventDisableTiming) != hipSuccess ||
      [&] {
        for (hipEvent_t& ev : e->tp_ev)
          if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return false;
        return true;
      }() == false ||
      hipStreamCreateWithFlags(&e->copy, hipStreamNonBlocking) != hipSuccess) {
    rg_destroy(e);
    return fail(RG_EHIP, "hipEventCreate / hipStreamCreate");
  }
  for (int b = 0; b < 2; ++b)
    if (hipEventCreateWithFlags(&e->a_gath[b], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->a_copy[b], hipEventDisableTiming) != hipSuccess) {
      rg_destroy(e);
      return fail(RG_EHIP, "hipEventCreate");
    }
  e->stream = e->own;
  std::vector<uint32_t> tab;
  build_crc(e, tab);
  if (hipMemcpy(e->crc_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    rg_destroy(e);
    return fail(RG_EHIP, "crc table upload");
  }
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c.device);
  const uint64_t per_cu = (uint64_t)std::max(bulk_blocks_per_cu(c.payload_bytes), 1);
  // bulk tiles: the largest power of two <= 64 replicas that still leaves a tile per resident wave
  // (r02 sweep, scripts/tile_sweep.sh: 64K x 3 picks 32, 1.160 -> 1.137 ms; C2 4,096 x 3 picks 2,
  // 0.094 -> 0.085 ms; the r01 rule asked for two tiles per wave and picked 16 and 1)
  const uint64_t waves = (uint64_t)std::max(cus, 1) * per_cu * 4;
  uint32_t tile = 64;
  while (tile > 1 && (n + tile - 1) / tile < waves) tile >>= 1;
#ifdef RG_AB_BULK_TILE  // A/B variant: a fixed tile (a power of two, 1..64)
  tile = RG_AB_BULK_TILE;
#endif
  e->bulk_tile = tile;
#ifdef RG_AB_APPLY_MEMCPY  // A/B variant: the runtime's hipMemcpyAsync for the copy-back's D2H leg
  e->copy_kernel = false;
#endif
  e->bulk_mj = c.max_entries_per_msg <= 16;
#ifdef RG_AB_CTL_FULL  // A/B variant: the full control step for every replica (no fast path)
  e->ctl_fast = false;
#endif
  // at most one wave per SIMD: occupancy buys nothing, and the fallback saves the slow kernel's launch
  e->ctl_fb = (uint64_t)n <= 64ull * 1024;
  if (const char* v = getenv("RAFTGPU_CTL_FB")) e->ctl_fb = v[0] == '1';  // test hook (both paths)
#ifdef RG_AB_BULK_MULTIJOB  // A/B variant: 0 / 1 forces the bulk kernel's job walk
  e->bulk_mj = RG_AB_BULK_MULTIJOB;
#endif
#ifdef RG_AB_NO_BULK_SMALL  // A/B variant: one-job replicas through bulk_kernel too
  e->bulk_small = false;
#endif
  {  // r05 turned these runtime A/B knobs into build variants (-DRG_AB_*, scripts/build_variant.sh): a script
     // still setting one would run the same build on both arms of its A/B, so say so once
    static bool warned = false;
    static const char* retired[] = {"RAFTGPU_BULK_MULTIJOB", "RAFTGPU_BULK_SMALL", "RAFTGPU_BULK_TILE",
                                    "RAFTGPU_BULK_GRID", "RAFTGPU_BULK_WG", "RAFTGPU_CTL_FAST", "RAFTGPU_WIRE_SIZING",
                                    "RAFTGPU_SYNC_DEBUG", "RAFTGPU_SMALL_GRID", "RAFTGPU_APPLY_MEMCPY", "RAFTGPU_POOL_PERM"};
    for (const char* k : retired)
      if (!warned && getenv(k)) {
        fprintf(stderr, "raftgpu: %s is no longer read (a build variant now: scripts/build_variant.sh -DRG_AB_...)\n", k);
        warned = true;
      }
  }
  if (const char* v = getenv("RAFTGPU_RCCL_SELF"))  // test hook: rg_wire_exchange's region to self moves too
    e->self_via_transport = !strcmp(v, "rccl");
  if (const char* v = getenv("RAFTGPU_APPLY_SDMA"))  // test hook: the SDMA D2H leg
    if (v[0] == '1') {
      std::string why;
      if (sdma_open(c.device, &e->sdma, &why) != 0) {
        rg_destroy(e);
        return fail(RG_EHIP, "RAFTGPU_APPLY_SDMA: " + why);
      }
    }
  if (launch_pool_reset(e->fring, e->npages, e->poolctl, e->stream) != hipSuccess ||
      hipStreamSynchronize(e->stream) != hipSuccess) {
    rg_destroy(e);
    return fail(RG_EHIP, "page pool reset");
  }
  const uint64_t ntiles = (n + tile - 1) / tile;
  // waves per bulk workgroup: the tiles of one group block's R slots are consecutive, so a workgroup
  // of R waves keeps a block's two followers — which read the same leader entries — on one CU and
  // one XCD's L2 (r04 A/B of 3 and 4 tied)
  e->bulk_wg = 4;
  const uint64_t wgw = e->bulk_wg;
  e->bulk_grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((ntiles + wgw - 1) / wgw,
                                                               (uint64_t)std::max(cus, 1) * per_cu * 4 / wgw));
#ifdef RG_AB_BULK_GRID  // A/B variant: a fixed bulk grid (blocks)
  e->bulk_grid = RG_AB_BULK_GRID;
#endif
  *out = e;
  return RG_OK;
}

void rg_destroy(rg_engine* e) {
  if (!e) return;
  if (e->sdma) sdma_close(e->sdma);
  for (int i = 0; i < 2; ++i) {
    if (e->gx[i]) (void)hipGraphExecDestroy(e->gx[i]);
    if (e->gg[i]) (void)hipGraphDestroy(e->gg[i]);
    if (e->g_ev[i]) {
      (void)hipEventSynchronize(e->g_ev[i]);
      (void)hipEventDestroy(e->g_ev[i]);
    }
  }
  if (e->g_htp) (void)hipHostFree(e->g_htp);
  if (e->own) {
    (void)hipStreamSynchronize(e->own);
    (void)hipStreamDestroy(e->own);
  }
  if (e->bulk) {
    (void)hipStreamSynchronize(e->bulk);
    (void)hipStreamDestroy(e->bulk);
  }
  for (hipEvent_t ev : e->ev_pool) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : e->ev_live) (void)hipEventDestroy(ev);
  for (int b = 0; b < 2; ++b) {
    if (e->ctl_done[b]) (void)hipEventDestroy(e->ctl_done[b]);
    if (e->bulk_done[b]) (void)hipEventDestroy(e->bulk_done[b]);
  }
  if (e->copy) {
    (void)hipStreamSynchronize(e->copy);
    (void)hipStreamDestroy(e->copy);
  }
  if (!e->hreg.empty()) {  // ranges the caller left registered
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    for (const auto& r : e->hreg) (void)hipHostUnregister((void*)r.first);
  }
  for (int b = 0; b < 2; ++b) {
    if (e->a_gath[b]) (void)hipEventDestroy(e->a_gath[b]);
    if (e->a_copy[b]) (void)hipEventDestroy(e->a_copy[b]);
    if (e->a_host[b]) (void)hipHostFree(e->a_host[b]);
  }
  if (e->ac_host) (void)hipHostFree(e->ac_host);
  if (e->pc_host) (void)hipHostFree(e->pc_host);
  if (e->stg_ev) (void)hipEventDestroy(e->stg_ev);
  if (e->rd_ev) (void)hipEventDestroy(e->rd_ev);
  if (e->cc_ev) (void)hipEventDestroy(e->cc_ev);
  if (e->h_cc) (void)hipHostFree(e->h_cc);
  if (e->h_rd) (void)hipHostFree(e->h_rd);
  if (e->prop_ev) (void)hipEventDestroy(e->prop_ev);
  for (hipEvent_t ev : e->tp_ev)
    if (ev) (void)hipEventDestroy(ev);
  if (e->h_tp) (void)hipHostFree(e->h_tp);
  if (e->h_fb) (void)hipHostFree(e->h_fb);
  for (void* p : e->allocs) (void)hipFree(p);
  if (e->h_bounds) (void)hipHostFree(e->h_bounds);
  if (e->h_need) (void)hipHostFree(e->h_need);
  for (hipEvent_t ev : e->need_ev)
    if (ev) (void)hipEventDestroy(ev);
  for (void* h : {(void*)e->h_pt, (void*)e->h_pc, (void*)e->h_hm, (void*)e->h_cmd, (void*)e->h_pcmd})
    if (h) (void)hipHostFree(h);
  delete e;
}

uint64_t rg_device_bytes(const rg_engine* e) { return e ? e->bytes : 0; }

int rg_probe_copy(int32_t device, uint64_t bytes, int32_t reps, double* gbps) {
  if (!gbps || bytes < 16 || reps < 1) return fail(RG_EINVAL, "rg_probe_copy args");
  HIPCHK(hipSetDevice(device));
  void *a = nullptr, *b = nullptr;
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = RG_OK;
  float best = 0;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) {
    rc = fail(RG_ENOMEM, "rg_probe_copy: hipMalloc");
  } else if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
             hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
    rc = fail(RG_EHIP, "rg_probe_copy: stream/events");
  } else {
    (void)hipMemsetAsync(a, 1, bytes, s);
    for (int r = 0; r <= reps && rc == RG_OK; ++r) {  // launch 0 warms up
      float ms = 0;
      if (hipEventRecord(e0, s) != hipSuccess || launch_probe_copy(a, b, bytes & ~15ull, s) != hipSuccess ||
          hipEventRecord(e1, s) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
          hipEventElapsedTime(&ms, e0, e1) != hipSuccess)
        rc = fail(RG_EHIP, "rg_probe_copy: launch");
      else if (r > 0 && (best == 0 || ms < best))
        best = ms;
    }
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (s) (void)hipStreamDestroy(s);
  if (a) (void)hipFree(a);
  if (b) (void)hipFree(b);
  if (rc == RG_OK) *gbps = 2.0 * (double)(bytes & ~15ull) / (best / 1e3) / 1e9;
  return rc;
}
uint64_t rg_tick_count(const rg_engine* e) { return e ? e->t : 0; }

int rg_set_stream(rg_engine* e, void* stream) {
  if (!e) return fail(RG_EINVAL, "null engine");
  hipStream_t ns = stream ? (hipStream_t)stream : e->own;
  if (ns != e->stream && e->stream) {  // keep tick order across the switch
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipStreamSynchronize(e->bulk));
  }
  e->stream = ns;
  return RG_OK;
}

// Make the engine's stream wait (on the device) for the last tick's bulk work.
static int join(rg_engine* e) {
  if (e->t > 0) HIPCHK(hipStreamWaitEvent(e->stream, e->bulk_done[(e->t - 1) & 1], 0));
  return RG_OK;
}

int rg_join(rg_engine* e) {
  if (!e) return fail(RG_EINVAL, "null engine");
  return join(e);
}

int rg_sync(rg_engine* e) {
  if (!e) return fail(RG_EINVAL, "null engine");
  int rc = join(e);
  if (rc) return rc;
  uint32_t perr = 0;
  HIPCHK(hipMemcpyAsync(&perr, &e->poolctl->param_err, 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (perr)
    return fail(RG_EINVARIANT, "control_kernel found a corrupt parameter block (checksum mismatch): a tick was skipped");
  return RG_OK;
}

int rg_bootstrap(rg_engine* e) {
  if (!e) return fail(RG_EINVAL, "null engine");
  HIPCHK(hipSetDevice(e->c.device));
  HIPCHK(hipStreamSynchronize(e->bulk));
  HIPCHK(hipStreamSynchronize(e->stream));
  e->t = 0;
  const uint64_t R = e->c.replicas, G = e->c.groups;
  for (int b = 0; b < 2; ++b) HIPCHK(hipMemsetAsync(e->cnt[b], 0, R * R * G * 4, e->stream));
  if (e->rcnt) HIPCHK(hipMemsetAsync(e->rcnt, 0, R * R * G * 4, e->stream));
  HIPCHK(hipMemsetAsync(e->feed, 0, (uint64_t)e->nrep * 8, e->stream));
  e->planned = e->wire_ready = false;
  e->recv = nullptr;
  RGCHK(stage_reset(e));
  for (uint64_t gi : e->touched) {
    e->h_pt[gi] = 0xFF;
    e->h_pc[gi] = 0;
    e->h_hm[gi] = 0;
    e->h_pcmd[gi] = make_uint2(0u, 0u);
  }
  e->touched.clear();
  e->staged = false;
  if (e->rd_reset_pending) HIPCHK(hipEventSynchronize(e->rd_ev));
  for (uint64_t i : e->rd_touched) e->h_rd[i] = 0;
  e->rd_touched.clear();
  if (e->cc_reset_pending) HIPCHK(hipEventSynchronize(e->cc_ev));
  for (uint64_t i : e->cc_touched) e->h_cc[i] = 0;
  e->cc_touched.clear();
  e->cc_staged = e->cc_reset_pending = false;
  e->rd_staged = e->rd_reset_pending = false;
  HIPCHK(hipMemsetAsync(e->rdst, 0, (uint64_t)RD_ROWS * e->nrep * 8, e->stream));
  HIPCHK(hipMemsetAsync(e->crc_err, 0, (uint64_t)e->nrep * 4, e->stream));
  HIPCHK(hipMemsetAsync(e->slow, 0, 8, e->stream));  // the fast path's hand-off counters
  HIPCHK(launch_pool_reset(e->fring, e->npages, e->poolctl, e->stream));  // every stream empty, every page free
  std::fill(e->cmd_used.begin(), e->cmd_used.end(), 0ull);
  std::fill(e->cmd_tick.begin(), e->cmd_tick.end(), ~0ull);
  TickParams p = params(e);
  for (int b = 0; b < 2; ++b) HIPCHK(hipMemsetAsync(e->jcnt[b], 0, (uint64_t)e->nrep * 4, e->stream));
  HIPCHK(launch_bootstrap(p, e->info, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return RG_OK;
}

int rg_fill_slabs(rg_engine* e) {
  if (!e) return fail(RG_EINVAL, "null engine");
  if (int jrc = join(e)) return jrc;
  HIPCHK(launch_fill_slabs(e->slabs, e->slab_info, 0, e->c.num_slabs, e->c.groups, e->slab_rows,
                           e->c.max_entries_per_msg, e->c.payload_bytes, e->c.seed, e->pl, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  e->slab_synth = ~0ull;
  return RG_OK;
}

// The host proposal tables still hold the batches the last tick uploaded: once that upload has
// completed, put the touched rows back to "no proposal".
static int stage_reset(rg_engine* e) {
  if (!e->stg_reset_pending) return RG_OK;
  HIPCHK(hipEventSynchronize(e->stg_ev));
  for (uint64_t gi : e->touched) {
    e->h_pt[gi] = 0xFF;
    e->h_pc[gi] = 0;
    e->h_hm[gi] = 0;
    e->h_pcmd[gi] = make_uint2(0u, 0u);
  }
  e->touched.clear();
  e->stg_reset_pending = false;
  return RG_OK;
}

// grow the caller-Cmd arenas (rare: a call's Cmds exceed a slab's arena): the old contents move
// with a synchronised device copy, since forwarded batches of the last ticks may still be read
static int cmd_reserve(rg_engine* e, uint64_t need_bytes) {
  if (need_bytes <= e->cmd_cap) return RG_OK;
  const uint64_t cap = std::max<uint64_t>((need_bytes * 3 / 2 + 4095) & ~4095ull, 1ull << 20);
  const uint32_t ns = e->c.num_slabs;
  uint8_t* nb = nullptr;
  RGCHK(dalloc(e, &nb, cap * ns));
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipStreamSynchronize(e->bulk));
  if (e->cmds) {
    for (uint32_t sl = 0; sl < ns; ++sl)
      if (e->cmd_used[sl])
        HIPCHK(hipMemcpy(nb + (uint64_t)sl * cap, e->cmds + (uint64_t)sl * e->cmd_cap, e->cmd_used[sl] * 16,
                         hipMemcpyDeviceToDevice));
    (void)hipFree(e->cmds);
    e->allocs.erase(std::remove(e->allocs.begin(), e->allocs.end(), (void*)e->cmds), e->allocs.end());
    e->bytes -= e->cmd_cap * ns;
  }
  e->cmds = nb;
  e->g_valid = false;  // captured bulk launches name the old arena
  e->cmd_cap = cap;
  return RG_OK;
}

// [p, p + n) inside one range the caller registered through rg_host_register
static bool host_registered(const rg_engine* e, const void* p, uint64_t n) {
  const uintptr_t a = (uintptr_t)p;
  for (const auto& r : e->hreg)
    if (a >= r.first && a + n <= r.first + r.second) return true;
  return false;
}

int rg_host_register(rg_engine* e, const void* p, size_t bytes) {
  if (!e || !p || !bytes) return fail(RG_EINVAL, "rg_host_register args");
  for (const auto& r : e->hreg)
    if ((uintptr_t)p < r.first + r.second && r.first < (uintptr_t)p + bytes)
      return fail(RG_EINVAL, "rg_host_register: overlaps a registered range");
  HIPCHK(hipSetDevice(e->c.device));
  HIPCHK(hipHostRegister(const_cast<void*>(p), bytes, hipHostRegisterDefault));
  e->hreg.emplace_back((uintptr_t)p, (uint64_t)bytes);
  return RG_OK;
}

int rg_host_unregister(rg_engine* e, const void* p) {
  if (!e || !p) return fail(RG_EINVAL, "rg_host_unregister args");
  for (size_t i = 0; i < e->hreg.size(); ++i)
    if (e->hreg[i].first == (uintptr_t)p) {
      if (int jrc = join(e)) return jrc;
      HIPCHK(hipStreamSynchronize(e->stream));  // no copy out of it is still in flight
      HIPCHK(hipHostUnregister(const_cast<void*>(p)));
      e->hreg.erase(e->hreg.begin() + i);
      return RG_OK;
    }
  return fail(RG_EINVAL, "rg_host_unregister: not a registered range");
}

int rg_propose(rg_engine* e, const rg_proposal* props, size_t n, const uint8_t* payload, const uint32_t* lens) {
  if (!e || (n && !props)) return fail(RG_EINVAL, "rg_propose args");
  RGCHK(stage_reset(e));
  const uint32_t N = e->pl.N, R = e->c.replicas, E = e->c.max_entries_per_msg, P = e->c.payload_bytes;
  const uint64_t g0 = (uint64_t)N * e->pl.col_base, gn = (uint64_t)N * e->c.groups;
  // validate every batch against the tables plus this call's earlier batches (all or nothing):
  // padd[input index] = this call's additions (count | slot << 8 | 1 << 16), cleared on the way out
  std::vector<uint32_t>& padd = e->padd;
  if (padd.size() < gn) padd.assign(gn, 0u);
  std::vector<uint64_t>& pset = e->pset;
  pset.clear();
  auto clear_add = [&] {
    for (uint64_t gi : pset) padd[gi] = 0;
    pset.clear();
  };
  uint64_t nent = 0, nbytes = 0;
  for (size_t i = 0; i < n; ++i) {
    const rg_proposal& b = props[i];
    if (b.group < g0 || b.group >= g0 + gn || b.slot >= R || b.count < 1 || b.count > E) {
      clear_add();
      return fail(RG_EINVAL, "rg_propose: batch " + std::to_string(i) + ": bad shard, slot or count");
    }
    if (pl_rank_of(e->pl, b.group, b.slot) != e->pl.rank) {
      clear_add();
      return fail(RG_EINVAL, "rg_propose: batch " + std::to_string(i) + ": that replica is hosted by another rank");
    }
    const uint64_t gi = b.group - g0;
    const uint32_t ad = padd[gi], added = ad & 0xFFu;
    const uint32_t have = e->h_pc[gi] + added;
    const uint32_t slot = ad ? (ad >> 8) & 0xFFu : e->h_pc[gi] ? e->h_pt[gi] : b.slot;
    if (have && slot != b.slot) {
      clear_add();
      return fail(RG_EFULL, "rg_propose: a second slot of one shard in one tick");
    }
    if (have + b.count > E) {
      clear_add();
      return fail(RG_EFULL, "rg_propose: batch larger than max_entries_per_msg");
    }
    if (!ad) pset.push_back(gi);
    padd[gi] = (added + b.count) | (b.slot << 8) | (1u << 16);
    nent = std::max<uint64_t>(nent, b.first + b.count);
  }
  clear_add();
  if (nent && !lens) return fail(RG_EINVAL, "rg_propose: null lens");
  for (uint64_t j = 0; j < nent; ++j) {
    if (lens[j] > e->maxc) return fail(RG_EINVAL, "rg_propose: Cmd longer than max_cmd_bytes");
    nbytes += lens[j];
  }
  if (nbytes && !payload) return fail(RG_EINVAL, "rg_propose: null payload");
  // the tick's slab: its Cmd arena restarts when a new tick takes it (stream order keeps the bytes of
  // the tick that used it nslab ticks ago until that tick and the next have read them)
  const uint64_t slab = e->t % e->c.num_slabs, rows = e->slab_rows;
  if (e->cmd_tick[slab] != e->t) {
    e->cmd_tick[slab] = e->t;
    e->cmd_used[slab] = 0;
  }
  // Layout: each Cmd at its own length rounded up to 16 B, back to back from cmd_used[slab], in batch
  // order. Per batch (host threads for a large call): its chunks, payload bytes, non-empty mask, the
  // chunk count all its Cmds share (~0u: none), and whether the caller's packing already is the arena's
  // (every Cmd but the last a multiple of 16 B: "flat"; the last one too: "aligned").
  PropScratch& ps = e->ps;
  ps.resize(n);
  const bool seq = [&] {  // batches name consecutive Cmds from lens[0]: payload offsets follow batch order
    uint64_t f = 0;
    for (size_t i = 0; i < n; ++i) {
      if (props[i].first != f) return false;
      f += props[i].count;
    }
    return true;
  }();
  auto batch_scan = [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      const rg_proposal& b = props[i];
      const uint32_t* L = lens + b.first;
      uint64_t ch = 0, by = 0, mk = 0;
      const uint32_t nc0 = (L[0] + 15) / 16;
      bool uni = true, flat = true;
      for (uint32_t x = 0; x < b.count; ++x) {
        const uint32_t ln = L[x], nc = (ln + 15) / 16;
        ch += nc;
        by += ln;
        mk |= (uint64_t)(ln != 0) << x;
        uni &= nc == nc0;
        if (x + 1 < b.count) flat &= (ln & 15u) == 0;
      }
      ps.ch[i] = ch;
      ps.by[i] = by;
      ps.mk[i] = mk;
      ps.nc0[i] = nc0;
      ps.fl[i] = (uint8_t)((uni ? 1 : 0) | (flat ? 2 : 0) | ((L[b.count - 1] & 15u) == 0 ? 4 : 0));
    }
  };
  const uint64_t T = n < 4096 ? 1 : std::min<uint64_t>({16, std::max(1u, std::thread::hardware_concurrency()), n / 2048});
  par_for(T, n, batch_scan);
  uint64_t chunks = 0;
  for (size_t i = 0; i < n; ++i) {
    ps.c0[i] = chunks;  // relative to a0 (added below)
    chunks += ps.ch[i];
  }
  // payload offset of each batch: by batch order (seq), else through the prefix over lens
  if (seq) {
    uint64_t o = 0;
    for (size_t i = 0; i < n; ++i) {
      ps.src[i] = o;
      o += ps.by[i];
    }
  } else {
    std::vector<uint64_t>& boff = e->pboff;
    boff.assign(nent + 1, 0);
    for (uint64_t j = 0; j < nent; ++j) boff[j + 1] = boff[j] + lens[j];
    for (size_t i = 0; i < n; ++i) ps.src[i] = boff[props[i].first];
  }
  const uint64_t a0 = e->cmd_used[slab];
  if (P && (a0 + chunks) >= SYN_OFF) return fail(RG_EFULL, "rg_propose: a slab's Cmd arena holds at most 32 GiB");
  if (P && chunks) RGCHK(cmd_reserve(e, (a0 + chunks) * 16));
  // the Cmd bytes move by DMA straight from the caller's buffer when it is registered
  // (rg_host_register) and falls into few runs; otherwise through pinned staging, in pieces whose
  // H2D copies overlap the host threads' copying of the next pieces
  const uint64_t cb = chunks * 16;
  uint64_t runs = 0;
  bool direct = false;
  if (P && cb && host_registered(e, payload, nbytes)) {
    direct = true;
    for (size_t i = 0; i < n && direct; ++i) {
      if (!(ps.fl[i] & 2)) direct = false;  // padding inside the batch: not the caller's packing
      if (i == 0 || !(ps.fl[i - 1] & 4) || ps.src[i] != ps.src[i - 1] + ps.by[i - 1]) ++runs;
    }
    if (runs > 1024) direct = false;
  }
  // pinned staging: [Cmd bytes (staged path) | per batch: info_at u64, first u64, chunk u32, count u32 | lens u32]
  const uint64_t sb = direct ? 0 : cb, dsc = n * 24, lb = (nent * 4 + 15) & ~15ull;
  const uint64_t need = sb + dsc + lb + 64;
  if (P && n) {
    HIPCHK(hipEventSynchronize(e->prop_ev));  // the last H2D out of h_cmd has completed
    if (need > e->h_cmd_cap) {
      if (e->h_cmd) (void)hipHostFree(e->h_cmd);
      e->h_cmd = nullptr;
      e->h_cmd_cap = 0;
      if (hipHostMalloc((void**)&e->h_cmd, need * 3 / 2, 0) != hipSuccess) return fail(RG_ENOMEM, "hipHostMalloc");
      e->h_cmd_cap = need * 3 / 2;
    }
    if (dsc + lb + 64 > e->d_cmd_cap) {
      HIPCHK(hipStreamSynchronize(e->stream));  // the last stage kernel read the old buffer
      if (e->d_cmd) {
        (void)hipFree(e->d_cmd);
        e->allocs.erase(std::remove(e->allocs.begin(), e->allocs.end(), (void*)e->d_cmd), e->allocs.end());
        e->bytes -= e->d_cmd_cap;
        e->d_cmd = nullptr;
      }
      e->d_cmd_cap = 0;
      RGCHK(dalloc(e, &e->d_cmd, (dsc + lb + 64) * 3 / 2));
      e->d_cmd_cap = (dsc + lb + 64) * 3 / 2;
    }
  }
  uint8_t* arena = P ? e->cmds + slab * e->cmd_cap : nullptr;
  // the host tables (serial over batches: a shard may come in several batches of one call)
  uint8_t* hd = e->h_cmd + sb;  // batch descriptors, then lens
  uint64_t* d_info = (uint64_t*)hd;
  uint64_t* d_first = d_info + n;
  uint32_t* d_chunk = (uint32_t*)(d_first + n);
  uint32_t* d_count = d_chunk + n;
  for (size_t i = 0; i < n; ++i) {
    const rg_proposal& b = props[i];
    const uint64_t gi = b.group - g0;
    const uint32_t j = (uint32_t)(b.group / N - e->pl.col_base);
    const uint64_t row = e->wire ? (uint64_t)b.slot * e->c.groups + j : j;
    const uint32_t at0 = e->h_pc[gi];  // position of the batch's first Cmd in the shard's batch
    if (P) {
      e->h_hm[gi] |= ps.mk[i] << at0;
      const uint32_t c0 = (uint32_t)(a0 + ps.c0[i]);
      uint2& pc = e->h_pcmd[gi];  // the shard's batch: chunks, contiguity, first arena chunk
      if (at0 == 0) {
        pc = make_uint2(1u << 31, c0);
        e->pnc[gi] = ps.nc0[i];
      }
      // contiguous while every Cmd has the first one's chunk count and follows the one before
      if (!(ps.fl[i] & 1) || ps.nc0[i] != e->pnc[gi] || (uint64_t)c0 != pc.y + (uint64_t)at0 * e->pnc[gi])
        pc.x &= ~(1u << 31);
      pc.x += (uint32_t)ps.ch[i];
      d_info[i] = (slab * rows + row) * E + at0;
      d_first[i] = b.first;
      d_chunk[i] = c0;
      d_count[i] = b.count;
    }
    if (!at0) e->touched.push_back(gi);
    e->h_pt[gi] = (uint8_t)b.slot;
    e->h_pc[gi] += b.count;
  }
  if (P && n) {
    uint32_t* hl = (uint32_t*)(hd + dsc);
    memcpy(hl, lens, nent * 4);
    if (direct) {
      // DMA straight from the caller's registered buffer, in stream order after the ticks that read
      // this slab last (the stage kernel after it zeroes the padding of short Cmds)
      for (size_t i = 0; i < n;) {
        size_t j = i;
        uint64_t by = ps.by[i];
        while (j + 1 < n && (ps.fl[j] & 4) && ps.src[j + 1] == ps.src[j] + ps.by[j]) by += ps.by[++j];
        if (by)
          HIPCHK(hipMemcpyAsync(arena + (a0 + ps.c0[i]) * 16, payload + ps.src[i], by, hipMemcpyHostToDevice, e->stream));
        i = j + 1;
      }
    } else if (cb) {
      // staged: pieces of about 64 MiB of the arena range; T threads copy each piece's batches (a
      // flat batch with one memcpy, any other Cmd by Cmd), and the H2D copy of a piece is issued as
      // soon as its batches are in, while the threads go on with the next piece
      std::vector<size_t>& pb = e->ppiece;  // first batch of each piece
      pb.clear();
      for (size_t i = 0; i < n; ++i)
        if (i == 0 || ps.c0[i] * 16 >= (ps.c0[pb.back()] * 16) + (64ull << 20)) pb.push_back(i);
      pb.push_back(n);
      const size_t np = pb.size() - 1;
      auto copy_batch = [&](size_t i) {
        const rg_proposal& b = props[i];
        uint8_t* d = e->h_cmd + ps.c0[i] * 16;
        const uint8_t* src = payload + ps.src[i];
        if (ps.fl[i] & 2) {
          if (ps.by[i]) memcpy(d, src, ps.by[i]);
          return;
        }
        for (uint32_t x = 0; x < b.count; ++x) {
          const uint32_t ln = lens[b.first + x];
          if (ln) memcpy(d, src, ln);
          d += (uint64_t)((ln + 15) / 16) * 16;
          src += ln;
        }
      };
      const uint64_t TT = std::min<uint64_t>({16, std::max(1u, std::thread::hardware_concurrency()), 1 + cb / (16ull << 20)});
      std::vector<std::atomic<uint32_t>> done(np);
      for (auto& d : done) d.store(0);
      auto worker = [&](uint64_t t) {
        for (size_t pc = 0; pc < np; ++pc) {
          const size_t lo = pb[pc], hi = pb[pc + 1], cnt = hi - lo;
          for (size_t i = lo + cnt * t / TT; i < lo + cnt * (t + 1) / TT; ++i) copy_batch(i);
          done[pc].fetch_add(1, std::memory_order_release);
        }
      };
      std::vector<std::thread> th;
      for (uint64_t t = 1; t < TT; ++t) th.emplace_back(worker, t);
      // the calling thread copies its share of each piece and issues the piece's H2D copy
      int herr = 0;
      for (size_t pc = 0; pc < np; ++pc) {
        const size_t lo = pb[pc], hi = pb[pc + 1], cnt = hi - lo;
        for (size_t i = lo; i < lo + cnt / TT; ++i) copy_batch(i);
        done[pc].fetch_add(1, std::memory_order_release);
        while (done[pc].load(std::memory_order_acquire) < TT) std::this_thread::yield();
        const uint64_t b0 = ps.c0[lo] * 16, b1 = hi < n ? ps.c0[hi] * 16 : cb;
        if (!herr && hipMemcpyAsync(arena + a0 * 16 + b0, e->h_cmd + b0, b1 - b0, hipMemcpyHostToDevice, e->stream) != hipSuccess)
          herr = 1;
      }
      for (auto& x : th) x.join();
      if (herr) return fail(RG_EHIP, "rg_propose: H2D copy of the staged Cmds failed");
    }
    HIPCHK(hipMemcpyAsync(e->d_cmd, hd, dsc + nent * 4, hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipEventRecord(e->prop_ev, e->stream));
    StageParams sp{};
    sp.slab_info = e->slab_info;
    sp.info_at = (const uint64_t*)e->d_cmd;
    sp.first = sp.info_at + n;
    sp.chunk = (const uint32_t*)(sp.first + n);
    sp.count = sp.chunk + n;
    sp.lens = (const uint32_t*)(e->d_cmd + dsc);
    sp.arena = arena;
    sp.n = n;
    LAUNCH(launch_stage_cmds(sp, e->stream), e->stream, "stage_cmds");
    e->cmd_used[slab] = a0 + chunks;
    e->slab_synth &= ~(1ull << slab);
    // "copied before return": the caller may reuse its buffer
    if (direct) HIPCHK(hipEventSynchronize(e->prop_ev));
  }
  if (n) e->staged = true;
  return RG_OK;
}

static int timing_event(rg_engine* e, hipStream_t s, int kind) {
  if (!(e->timing & (1 << kind)) || e->t % e->timing_every) return RG_OK;
  hipEvent_t ev;
  if (e->ev_pool.empty()) {
    // timing only: no system-scope fence (its L2 writeback and invalidate cost the timed tick ~3 %,
    // r04k: 1.342 ms with events on one tick in four against 1.299 ms without)
    HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableSystemFence));
  } else {
    ev = e->ev_pool.back();
    e->ev_pool.pop_back();
  }
  e->ev_live.push_back(ev);
  if (e->ev_live.size() & 1) {
    e->ev_kind.push_back(kind);
    e->ev_tick.push_back(e->t);
  }
  HIPCHK(hipEventRecord(ev, s));
  return RG_OK;
}

// rg_timing_epoch: one reference event per process (the device's timeline origin for every engine)
static hipEvent_t g_epoch = nullptr;
static int g_epoch_dev = -1;

static int timing_drain(rg_engine* e) {
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipStreamSynchronize(e->bulk));
  const bool epoch = g_epoch && g_epoch_dev == e->c.device;
  for (size_t i = 0; i + 1 < e->ev_live.size(); i += 2) {
    float ms = 0;
    const int k = e->ev_kind[i / 2];
    HIPCHK(hipEventElapsedTime(&ms, e->ev_live[i], e->ev_live[i + 1]));
    e->kms[k] += ms;
    e->klaunch[k]++;
    if (epoch) {
      float a = 0, b = 0;
      HIPCHK(hipEventElapsedTime(&a, g_epoch, e->ev_live[i]));
      HIPCHK(hipEventElapsedTime(&b, g_epoch, e->ev_live[i + 1]));
      e->kev[k].push_back({e->ev_tick[i / 2], (double)a, (double)b});
    }
  }
  e->ev_kind.clear();
  e->ev_tick.clear();
  e->ev_pool.insert(e->ev_pool.end(), e->ev_live.begin(), e->ev_live.end());
  e->ev_live.clear();
  return RG_OK;
}

int rg_timing(rg_engine* e, int enable) {
  if (!e) return fail(RG_EINVAL, "null engine");
  if (int rc = timing_drain(e)) return rc;
  // 1: both kernels (4 event records per tick), 2: bulk_kernel only (2 per tick); bits 8..: time
  // every n-th tick only (each timed event record costs the tick about 50 µs on this runtime, r03d)
  const int mode = enable & 0xFF, every = enable >> 8;
  e->timing = mode == 1 ? 3 : mode == 2 ? 2 : 0;
  e->timing_every = every > 0 ? (uint32_t)every : 1u;
  e->kms[0] = e->kms[1] = 0;
  e->klaunch[0] = e->klaunch[1] = 0;
  e->kev[0].clear();
  e->kev[1].clear();
  return RG_OK;
}

int rg_timing_epoch(int device) {
  HIPCHK(hipSetDevice(device));
  if (g_epoch && g_epoch_dev != device) {
    (void)hipEventDestroy(g_epoch);
    g_epoch = nullptr;
  }
  if (!g_epoch) HIPCHK(hipEventCreate(&g_epoch));
  HIPCHK(hipDeviceSynchronize());  // every event recorded later lies after it on the device's timeline
  HIPCHK(hipEventRecord(g_epoch, nullptr));
  HIPCHK(hipEventSynchronize(g_epoch));
  g_epoch_dev = device;
  return RG_OK;
}

int rg_kernel_events(rg_engine* e, int kernel, uint64_t* ticks, double* start_ms, double* end_ms, uint64_t cap,
                     uint64_t* n) {
  if (!e || !n || kernel < 0 || kernel > 1 || (cap && (!ticks || !start_ms || !end_ms)))
    return fail(RG_EINVAL, "rg_kernel_events args");
  if (int rc = timing_drain(e)) return rc;
  const auto& v = e->kev[kernel];
  *n = v.size();
  for (uint64_t i = 0; i < cap && i < v.size(); ++i) {
    ticks[i] = v[i].tick;
    start_ms[i] = v[i].start;
    end_ms[i] = v[i].end;
  }
  return RG_OK;
}

int rg_kernel_ms(rg_engine* e, double* ms, uint64_t* launches) {
  if (!e || !ms || !launches) return fail(RG_EINVAL, "rg_kernel_ms args");
  if (int rc = timing_drain(e)) return rc;
  for (int k = 0; k < 2; ++k) {
    ms[k] = e->kms[k];
    launches[k] = e->klaunch[k];
  }
  return RG_OK;
}

// control_kernel(t) reads its parameter block from a device slot written by a copy on the same
// stream just before the launch, so the launch's own kernel arguments are one pointer
// the checksum the kernel verifies before it dereferences anything
static void seal(TickParams& p) {
  uint64_t w[TP_WORDS], h = 0;
  memcpy(w, &p, sizeof w);
  for (uint32_t i = 0; i < TP_WORDS; ++i) h += tp_term(w[i], i);
  p.csum = h;
}

// the fields tick_impl sets from the tick's inputs and staging (the rest follows from the tick number)
static void copy_inputs(TickParams& d, const TickParams& s) {
  d.flags = s.flags;
  d.prop_target = s.prop_target; d.prop_count = s.prop_count; d.prop_hmask = s.prop_hmask; d.prop_cmd = s.prop_cmd;
  d.campaign = s.campaign; d.isolate = s.isolate; d.read_ctx = s.read_ctx; d.cc_in = s.cc_in;
}

// The tick's parameter block reaches its device slot before the control launch, in stream order. A
// copy is a blit kernel of ~5 µs on the GPU's timeline (a quarter of a metadata-only C2 tick), so a
// chunk's first tick copies TP_CHUNK blocks at once — its own and the next ticks' as they will be if
// their inputs stay the same (the steady state: rg_tick_device with the same device inputs) — and a
// later tick copies only when its block differs from the speculated one. The kernel checks every
// block's checksum either way (tp_verify).
static int launch_control_slot(rg_engine* e, const TickParams& p) {
  const uint32_t k = (uint32_t)(e->tp_next++ % TP_SLOTS), c = k / TP_CHUNK;
  TickParams blk = p;
  seal(blk);
  if (e->tp_corrupt) {  // tests only: a torn block, as a stale kernel-argument line would look
    e->tp_corrupt--;
    blk.csum ^= 0x100ull;
  }
  if (k % TP_CHUNK == 0) {
    if (e->tp_used[c]) HIPCHK(hipEventSynchronize(e->tp_ev[c]));
    e->h_tp[k] = blk;
    for (uint32_t i = 1; i < TP_CHUNK; ++i) {
      TickParams s = params_at(e, p.tick + i);
      copy_inputs(s, p);
      seal(s);
      e->h_tp[k + i] = s;
    }
    HIPCHK(hipMemcpyAsync(e->d_tp + k, e->h_tp + k, TP_CHUNK * sizeof(TickParams), hipMemcpyHostToDevice, e->stream));
    e->tp_copies++;
  } else if (memcmp(&e->h_tp[k], &blk, sizeof(TickParams)) != 0) {
    e->h_fb[k] = blk;
    HIPCHK(hipMemcpyAsync(e->d_tp + k, e->h_fb + k, sizeof(TickParams), hipMemcpyHostToDevice, e->stream));
    e->tp_copies++;
  }
  if (k % TP_CHUNK == TP_CHUNK - 1) {
    HIPCHK(hipEventRecord(e->tp_ev[c], e->stream));
    e->tp_used[c] = true;
  }
  if (e->ctl_fast)
    LAUNCH(launch_control_fast(e->d_tp + k, &e->poolctl->param_err, p.R, p.nrep, e->ctl_fb, e->stream), e->stream,
           "control_fast_kernel / control_slow_kernel");
  else
    LAUNCH(launch_control(e->d_tp + k, &e->poolctl->param_err, p.R, p.nrep, e->stream), e->stream, "control_kernel");
  return RG_OK;
}

static int tick_impl(rg_engine* e, const rg_tick_input* in, bool device_ptrs) {
  if (e->wire && e->t > 0 && !e->wire_ready)
    return fail(RG_EINVAL, "rg_tick: the last tick's messages were not exchanged (rg_wire_plan/pack/recv)");
  TickParams p = params(e);
  if (e->staged && in && in->prop_target)
    return fail(RG_EINVAL, "rg_tick: proposals staged by rg_propose and tick-input proposals in one tick");
  const uint32_t sl = (uint32_t)(e->t % e->c.num_slabs);
  if (in && in->prop_target && !((e->slab_synth >> sl) & 1) && e->c.payload_bytes) {
    // a tick-input (synthetic) batch into a slab rg_propose wrote: regenerate that slab only (the
    // others may still hold forwarded proposals' Cmds)
    LAUNCH(launch_fill_slabs(e->slabs, e->slab_info, sl, 1, e->c.groups, e->slab_rows, e->c.max_entries_per_msg,
                             e->c.payload_bytes, e->c.seed, e->pl, e->stream),
           e->stream, "fill_slabs");
    e->slab_synth |= 1ull << sl;
  }
  if (in) {
    p.flags = in->flags;
    if (device_ptrs) {
      if (in->prop_target && !in->prop_count) return fail(RG_EINVAL, "prop_target without prop_count");
      p.prop_target = in->prop_target;
      p.prop_count = in->prop_count;
      p.campaign = in->campaign;
      p.isolate = in->isolate;
    } else {
      const uint64_t G = (uint64_t)e->c.groups * e->pl.N, n = G * e->c.replicas;  // global inputs
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
  if (e->staged) {  // rg_propose's batches: upload the tables (pinned; reset once the copy completed)
    const uint64_t GN = (uint64_t)e->c.groups * e->pl.N;
    HIPCHK(hipMemcpyAsync(e->d_prop_target, e->h_pt, GN, hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipMemcpyAsync(e->d_prop_count, e->h_pc, GN * 4, hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipMemcpyAsync(e->d_prop_hmask, e->h_hm, GN * 8, hipMemcpyHostToDevice, e->stream));
    if (e->c.payload_bytes) {
      HIPCHK(hipMemcpyAsync(e->d_prop_cmd, e->h_pcmd, GN * 8, hipMemcpyHostToDevice, e->stream));
      p.prop_cmd = e->d_prop_cmd;
    }
    HIPCHK(hipEventRecord(e->stg_ev, e->stream));
    p.prop_target = e->d_prop_target;
    p.prop_count = e->d_prop_count;
    p.prop_hmask = e->d_prop_hmask;
    e->staged = false;
    e->stg_reset_pending = true;
  }
  if (e->rd_staged) {  // rg_read_index's requests
    HIPCHK(hipMemcpyAsync(e->d_read_ctx, e->h_rd, (uint64_t)e->nrep * e->pl.N * 8, hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipEventRecord(e->rd_ev, e->stream));
    p.read_ctx = e->d_read_ctx;
    e->rd_staged = false;
    e->rd_reset_pending = true;
  }
  if (e->cc_staged) {  // rg_config_change's membership changes
    HIPCHK(hipMemcpyAsync(e->d_cc, e->h_cc, (uint64_t)e->c.groups * e->pl.N * 2, hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipEventRecord(e->cc_ev, e->stream));
    p.cc_in = e->d_cc;
    e->cc_staged = false;
    e->cc_reset_pending = true;
  }
  // control(t) on the engine stream once bulk(t-2) released jobs[t&1]; bulk(t) on the bulk
  // stream after control(t). control(t+1) then overlaps bulk(t): they touch disjoint data.
  const int a = (int)(e->t & 1);
#ifdef RG_OVERLAP  // ablation: bulk(t) on a second stream beside control(t+1)
  hipStream_t bs = e->bulk;
#else  // measured r01: beside bulk the latency-bound control kernel ran 8x slower, a net loss
  hipStream_t bs = e->stream;
#endif
  // One stream (the product): stream order alone sequences control and bulk, so no event
  // records or waits go between them (each is a packet in the queue, ≈5 µs a tick at 4K groups).
  // (r03: bulk_done, which only orders a second stream, is no longer recorded every tick either;
  // rg_set_stream synchronises before it switches streams.)
  const bool two = bs != e->stream;
  if (two && e->t >= 2) HIPCHK(hipStreamWaitEvent(e->stream, e->bulk_done[a], 0));
  RGCHK(timing_event(e, e->stream, 0));
  RGCHK(launch_control_slot(e, p));
  if (e->c.payload_bytes) {  // stream pages: release what compaction passed, take what this step's appends need
    PoolParams pp{};
    pp.nrep = e->nrep; pp.PTS = e->PTS; pp.npages = e->npages;
    pp.s32 = p.s32; pp.pt = e->pt; pp.fring = e->fring; pp.ctl = e->poolctl;
    pp.jcnt = p.jcnt;
    LAUNCH(launch_pool(pp, e->stream), e->stream, "pool_kernel");
  }
  RGCHK(timing_event(e, e->stream, 0));
  if (two) {
    HIPCHK(hipEventRecord(e->ctl_done[a], e->stream));
    HIPCHK(hipStreamWaitEvent(bs, e->ctl_done[a], 0));
  }
  // metadata-only engines (P = 0) have no payload stage: every reader of an entry takes its type
  // from the term word and its CRC is 0 (no Cmd bytes), so no info word needs writing and the tick
  // is the control launch alone
  if (e->c.payload_bytes) {
    RGCHK(timing_event(e, bs, 1));
    LAUNCH(launch_bulk(bulk_params(e), e->pt, bs, e->bulk_grid), bs, "bulk_kernel");
    RGCHK(timing_event(e, bs, 1));
  }
  // bulk_done orders other streams behind the payload stage (join, the overlap ablation); with one
  // stream, stream order already does, and an event record is one more packet per tick
  if (two) HIPCHK(hipEventRecord(e->bulk_done[a], bs));
  e->t++;
  e->wire_ready = false;
  if (!device_ptrs && in) HIPCHK(hipStreamSynchronize(e->stream));  // host buffers may be reused
  return RG_OK;
}

int rg_tick(rg_engine* e, const rg_tick_input* in) {
  if (!e) return fail(RG_EINVAL, "null engine");
  return tick_impl(e, in, false);
}

// ---- the multi-tick path: k ticks with the same device-resident inputs. With
// RG_TICKN_GRAPH the k ticks are one captured HIP graph — per tick a parameter-slot copy and the
// control / pool / bulk launches — replayed with one hipGraphLaunch; the host writes the k parameter
// blocks into the graph's pinned slots before each launch (the copy nodes read them when they run).
static int tick_graph(rg_engine* e, const rg_tick_input* in, uint32_t k) {
  const uint64_t t0 = e->t;
  const bool same = e->g_valid && e->g_k == k && e->g_par == (uint32_t)(t0 & 1) && e->g_stream == e->stream &&
                    !memcmp(&e->g_in, in, sizeof *in);
  if (!same) {
    HIPCHK(hipStreamSynchronize(e->stream));
    for (int i = 0; i < 2; ++i) {
      if (e->gx[i]) (void)hipGraphExecDestroy(e->gx[i]);
      if (e->gg[i]) (void)hipGraphDestroy(e->gg[i]);
      e->gx[i] = nullptr;
      e->gg[i] = nullptr;
      e->g_used[i] = false;
    }
    e->g_valid = false;
    if (!e->g_dtp) {
      RGCHK(dalloc(e, &e->g_dtp, 2ull * G_MAXK * sizeof(TickParams)));
      if (hipHostMalloc((void**)&e->g_htp, 2ull * G_MAXK * sizeof(TickParams), 0) != hipSuccess)
        return fail(RG_ENOMEM, "hipHostMalloc (graph parameter slots)");
      for (int i = 0; i < 2; ++i) HIPCHK(hipEventCreateWithFlags(&e->g_ev[i], hipEventDisableTiming));
    }
    for (int set = 0; set < 2; ++set) {
      HIPCHK(hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
      // every path out of the capture ends it: a failed launch leaves the stream usable
      // and reports its own error, not a later capture-invalidated one
      auto capture = [&]() -> hipError_t {
      for (uint32_t i = 0; i < k; ++i) {
        TickParams p = params_at(e, t0 + i);
        p.flags = in->flags;
        p.prop_target = in->prop_target;
        p.prop_count = in->prop_count;
        p.campaign = in->campaign;
        p.isolate = in->isolate;
        TickParams* hs = e->g_htp + set * G_MAXK + i;
        TickParams* ds = e->g_dtp + set * G_MAXK + i;
        hipError_t r = hipMemcpyAsync(ds, hs, sizeof(TickParams), hipMemcpyHostToDevice, e->stream);
        if (r == hipSuccess)
          r = e->ctl_fast ? launch_control_fast(ds, &e->poolctl->param_err, p.R, p.nrep, e->ctl_fb, e->stream)
                          : launch_control(ds, &e->poolctl->param_err, p.R, p.nrep, e->stream);
        if (r == hipSuccess && e->c.payload_bytes) {
          PoolParams pp{};
          pp.nrep = e->nrep; pp.PTS = e->PTS; pp.npages = e->npages;
          pp.s32 = p.s32; pp.pt = e->pt; pp.fring = e->fring; pp.ctl = e->poolctl;
          pp.jcnt = p.jcnt;
          r = launch_pool(pp, e->stream);
          if (r == hipSuccess) r = launch_bulk(bulk_params_at(e, t0 + i), e->pt, e->stream, e->bulk_grid);
        }
        if (r != hipSuccess) return r;
      }
      return hipSuccess;
      };
      const hipError_t cr = capture();
      hipError_t r = hipStreamEndCapture(e->stream, &e->gg[set]);
      if (cr != hipSuccess) {
        if (r == hipSuccess && e->gg[set]) (void)hipGraphDestroy(e->gg[set]);
        e->gg[set] = nullptr;
        return fail(RG_EHIP, std::string("rg_tick_device_n: graph capture: ") + hipGetErrorString(cr));
      }
      if (r != hipSuccess) return fail(RG_EHIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(r));
      HIPCHK(hipGraphInstantiate(&e->gx[set], e->gg[set], nullptr, nullptr, 0));
    }
    e->g_k = k;
    e->g_par = (uint32_t)(t0 & 1);
    e->g_stream = e->stream;
    e->g_in = *in;
    e->g_flip = 0;
    e->g_valid = true;
  }
  const uint32_t set = e->g_flip;
  if (e->g_used[set]) HIPCHK(hipEventSynchronize(e->g_ev[set]));  // its copy nodes have read the slots
  for (uint32_t i = 0; i < k; ++i) {
    TickParams p = params_at(e, t0 + i);
    p.flags = in->flags;
    p.prop_target = in->prop_target;
    p.prop_count = in->prop_count;
    p.campaign = in->campaign;
    p.isolate = in->isolate;
    seal(p);
    e->g_htp[set * G_MAXK + i] = p;
  }
  HIPCHK(hipGraphLaunch(e->gx[set], e->stream));
  HIPCHK(hipEventRecord(e->g_ev[set], e->stream));
  e->g_used[set] = true;
  e->g_flip ^= 1u;
  e->t += k;
  HIPCHK(hipEventRecord(e->bulk_done[(e->t - 1) & 1], e->stream));
  return RG_OK;
}

// RG_TICKN_RESIDENT: the k ticks of a metadata-only one-rank engine in ONE launch of the resident
// control kernel (a workgroup per 64 groups holding all their replicas, a barrier between ticks)
static int tick_resident(rg_engine* e, const rg_tick_input* in, uint32_t k) {
  if (!e->g_dtp) {
    RGCHK(dalloc(e, &e->g_dtp, 2ull * G_MAXK * sizeof(TickParams)));
    if (hipHostMalloc((void**)&e->g_htp, 2ull * G_MAXK * sizeof(TickParams), 0) != hipSuccess)
      return fail(RG_ENOMEM, "hipHostMalloc (graph parameter slots)");
    for (int i = 0; i < 2; ++i) HIPCHK(hipEventCreateWithFlags(&e->g_ev[i], hipEventDisableTiming));
  }
  const uint32_t set = e->g_flip;
  if (e->g_used[set]) HIPCHK(hipEventSynchronize(e->g_ev[set]));  // its copy has read the slots
  for (uint32_t i = 0; i < k; ++i) {
    TickParams p = params_at(e, e->t + i);
    p.flags = in->flags;
    p.prop_target = in->prop_target;
    p.prop_count = in->prop_count;
    p.campaign = in->campaign;
    p.isolate = in->isolate;
    seal(p);
    e->g_htp[set * G_MAXK + i] = p;
  }
  TickParams* ds = e->g_dtp + set * G_MAXK;
  HIPCHK(hipMemcpyAsync(ds, e->g_htp + set * G_MAXK, k * sizeof(TickParams), hipMemcpyHostToDevice, e->stream));
  HIPCHK(hipEventRecord(e->g_ev[set], e->stream));
  LAUNCH(launch_control_resident(ds, k, &e->poolctl->param_err, e->c.replicas, e->c.groups, e->stream), e->stream,
         "control_resident_kernel");
  e->g_used[set] = true;
  e->g_flip ^= 1u;
  e->g_valid = false;  // the graph path's slots were reused
  e->t += k;
  return RG_OK;
}

int rg_tick_device_n(rg_engine* e, const rg_tick_input* in, uint32_t k, uint32_t flags) {
  if (!e || !in || k == 0 || (flags & ~(RG_TICKN_GRAPH | RG_TICKN_RESIDENT)) ||
      (flags & RG_TICKN_GRAPH && flags & RG_TICKN_RESIDENT))
    return fail(RG_EINVAL, "rg_tick_device_n args");
  if (in->prop_target && !in->prop_count) return fail(RG_EINVAL, "prop_target without prop_count");
  if (flags & RG_TICKN_RESIDENT) {
    if (e->c.payload_bytes || e->wire || e->c.replicas > 4 || k > G_MAXK || e->staged || e->rd_staged ||
        e->cc_staged || e->timing)
      return fail(RG_EINVAL, "rg_tick_device_n: resident ticks need a metadata-only one-rank engine with at most 4 "
                             "replicas, nothing staged, timing off, k <= 64");
    HIPCHK(hipSetDevice(e->c.device));
    return tick_resident(e, in, k);
  }
  if (!(flags & RG_TICKN_GRAPH)) {
    for (uint32_t i = 0; i < k; ++i) RGCHK(tick_impl(e, in, true));
    return RG_OK;
  }
  const uint32_t ns = e->c.num_slabs, period = ns % 2 ? 2 * ns : ns;
  if (k > G_MAXK || k % period)
    return fail(RG_EINVAL, "rg_tick_device_n: a graph runs a multiple of lcm(2, num_slabs) ticks, at most 64");
  if (e->wire || e->staged || e->rd_staged || e->cc_staged || e->timing)
    return fail(RG_EINVAL, "rg_tick_device_n: graphs need a one-rank engine with nothing staged and timing off");
  HIPCHK(hipSetDevice(e->c.device));
  if (in->prop_target && e->c.payload_bytes) {
    // tick-input batches carry generator Cmds: regenerate every slab rg_propose wrote, as tick_impl
    // would when a tick-input batch takes it — except the last tick's, whose forwarded batches the
    // first graph tick may still read (then one plain tick first)
    const uint64_t prev = e->t ? (e->t - 1) % ns : ~0ull;
    for (uint32_t sl = 0; sl < ns; ++sl) {
      if ((e->slab_synth >> sl) & 1) continue;
      if (sl == prev) return fail(RG_EINVAL, "rg_tick_device_n: the last tick's slab holds caller Cmds (tick once first)");
      LAUNCH(launch_fill_slabs(e->slabs, e->slab_info, sl, 1, e->c.groups, e->slab_rows, e->c.max_entries_per_msg,
                               e->c.payload_bytes, e->c.seed, e->pl, e->stream),
             e->stream, "fill_slabs");
      e->slab_synth |= 1ull << sl;
    }
  }
  return tick_graph(e, in, k);
}

int rg_tick_device(rg_engine* e, const rg_tick_input* in) {
  if (!e) return fail(RG_EINVAL, "null engine");
  return tick_impl(e, in, true);
}

int rg_read_replicas(rg_engine* e, uint32_t first, uint32_t n, rg_replica_view* out) {
  if (!e || !out || (uint64_t)first + n > e->nrep) return fail(RG_EINVAL, "rg_read_replicas range");
  if (int jrc = join(e)) return jrc;
  if (n == 0) return RG_OK;
  int rc = stage_reserve(e, (uint64_t)n * sizeof(rg_replica_view));
  if (rc) return rc;
  HIPCHK(launch_gather_replicas(admin(e), first, n, e->stage, e->stream));
  HIPCHK(hipMemcpyAsync(out, e->stage, (uint64_t)n * sizeof(rg_replica_view), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return RG_OK;
}

int rg_read_msgs(rg_engine* e, uint32_t rid, uint32_t dst, rg_msg_view* out, uint32_t cap, uint64_t* terms) {
  if (!e || rid >= e->nrep || dst >= e->c.replicas) return fail(RG_EINVAL, "rg_read_msgs range");
  if (int jrc = join(e)) return jrc;
  const uint32_t K = e->c.max_msgs_per_pair, E = e->c.max_entries_per_msg;
  const uint64_t hb = (uint64_t)K * 64, tb = (uint64_t)K * E * 8;
  int rc = stage_reserve(e, hb + tb + 16);
  if (rc) return rc;
  uint8_t* d = e->stage;
  HIPCHK(launch_gather_msgs(admin(e), rid, dst, d, (uint64_t*)(d + hb), (uint32_t*)(d + hb + tb), e->stream));
  std::vector<uint8_t> h(hb + tb + 4);
  HIPCHK(hipMemcpyAsync(h.data(), d, h.size(), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  uint32_t n = 0;
  memcpy(&n, h.data() + hb + tb, 4);
  const uint32_t m = std::min(std::min(n, cap), K);
  if (out && m) memcpy(out, h.data(), (uint64_t)m * sizeof(rg_msg_view));
  if (terms && m) memcpy(terms, h.data() + hb, (uint64_t)m * E * 8);
  return (int)n;
}

int rg_read_entries(rg_engine* e, uint32_t rid, uint64_t first, uint32_t n, rg_entry_view* out, uint8_t* payload) {
  if (!e || rid >= e->nrep || !out) return fail(RG_EINVAL, "rg_read_entries args");
  if (n == 0) return RG_OK;
  rg_replica_view v;
  int rc = rg_read_replicas(e, rid, 1, &v);
  if (rc) return rc;
  if (first <= v.marker || first + n - 1 > v.last) return fail(RG_EINVAL, "index outside (marker, last]");
  const uint64_t vb = a16((uint64_t)n * sizeof(rg_entry_view));
  RGCHK(stage_reserve(e, vb + 16));
  HIPCHK(launch_gather_entries(admin(e), rid, first, n, e->stage, e->stream));
  HIPCHK(hipMemcpyAsync(out, e->stage, (uint64_t)n * sizeof(rg_entry_view), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (!payload) return RG_OK;
  // the Cmds, packed back to back in entry order at their own lengths: gathered 16-B aligned into
  // device staging, one D2H copy, then packed on the host
  std::vector<uint64_t> ao(n, ~0ull);
  uint64_t tot = 0;
  for (uint32_t i = 0; i < n; ++i)
    if (out[i].type == RG_ENTRY_APPLICATION && out[i].len) {
      ao[i] = tot;
      tot += a16(out[i].len);
    }
  if (!tot) return RG_OK;
  const uint64_t ob = a16((uint64_t)n * 8);
  RGCHK(stage_reserve(e, ob + tot + 16));
  HIPCHK(hipMemcpyAsync(e->stage, ao.data(), (uint64_t)n * 8, hipMemcpyHostToDevice, e->stream));
  HIPCHK(launch_gather_cmds(admin(e), rid, first, n, (const uint64_t*)e->stage, e->stage + ob, e->stream));
  std::vector<uint8_t> host(tot);
  HIPCHK(hipMemcpyAsync(host.data(), e->stage + ob, tot, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  uint64_t at = 0;
  for (uint32_t i = 0; i < n; ++i)
    if (ao[i] != ~0ull) {
      memcpy(payload + at, host.data() + ao[i], out[i].len);
      at += out[i].len;
    }
  return RG_OK;
}

int rg_import_replica(rg_engine* e, uint32_t rid, const rg_replica_view* v, const uint64_t* terms,
                      const uint32_t* types, const uint8_t* payloads, const uint32_t* lens) {
  if (!e || !v || rid >= e->nrep) return fail(RG_EINVAL, "rg_import_replica args");
  if (int jrc = join(e)) return jrc;
  const uint64_t L = e->c.log_capacity, P = e->c.payload_bytes, row = e->maxc;
  if (v->last < v->marker || v->last - v->marker > L) return fail(RG_EINVAL, "log longer than the ring");
  if (v->term > TERM_MASK || v->marker_term > TERM_MASK || v->snap_term > TERM_MASK)
    return fail(RG_EINVAL, "rg_import_replica: term >= 2^36 (the term word's field, DESIGN.md §2)");
  const uint32_t nent = (uint32_t)(v->last - v->marker);
  if (nent && !terms) return fail(RG_EINVAL, "rg_import_replica: null terms");
  std::vector<uint64_t> words(nent);
  std::vector<uint32_t> crcs(nent, 0), pos(nent, 0);
  std::vector<uint8_t> chunks;  // the Cmds back to back, each zero-padded to whole chunks (a fresh stream)
  std::vector<uint8_t> slot;
  uint64_t src = 0;  // the caller's Cmds are packed back to back (one per entry with a Cmd)
  for (uint32_t k = 0; k < nent; ++k) {
    const uint32_t type = types ? (types[k] & 0xFFu) : RG_ENTRY_APPLICATION;
    const uint32_t len = lens ? lens[k] : (uint32_t)P;
    pos[k] = (uint32_t)(chunks.size() / 16);
    if (terms[k] > TERM_MASK) return fail(RG_EINVAL, "rg_import_replica: term >= 2^36");
    if (type != RG_ENTRY_APPLICATION) {  // a ConfigChange keeps its descriptor, no Cmd
      const uint32_t cc = lens ? lens[k] : 0u;
      if (cc > 0xFFu) return fail(RG_EINVAL, "rg_import_replica: ConfigChange descriptor out of range");
      words[k] = (terms[k] & TERM_MASK) | TYPE_BIT | cc_bits(cc);
      continue;
    }
    if (len > row) return fail(RG_EINVAL, "rg_import_replica: Cmd longer than max_cmd_bytes");
    const bool hp = payloads && P && len && !(types && (types[k] & RG_ENTRY_EMPTY));
    words[k] = (terms[k] & TERM_MASK) | (hp ? len_bits(len) : 0);
    if (hp) {
      const uint64_t S = (len + P - 1) / P;  // the slot CRC: the Cmd zero-padded to S·P bytes
      slot.assign(S * P, 0);
      memcpy(slot.data(), payloads + src, len);
      src += len;
      crcs[k] = host_crc(e, slot.data(), S * P);
      chunks.insert(chunks.end(), slot.begin(), slot.begin() + (len + 15) / 16 * 16);
    }
  }
  const uint64_t nch = chunks.size() / 16;
  if (nch && vpn_ceil((uint32_t)nch) > e->PTS) return fail(RG_EFULL, "rg_import_replica: log longer than stream_pages");
  const uint64_t vb = 512, wb = (uint64_t)nent * 8, cb = (uint64_t)nent * 4, pb = chunks.size();
  int rc = stage_reserve(e, vb + wb + 2 * cb + pb + 64);
  if (rc) return rc;
  uint8_t* d = e->stage;
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipMemcpy(d, v, sizeof *v, hipMemcpyHostToDevice));
  if (wb) HIPCHK(hipMemcpy(d + vb, words.data(), wb, hipMemcpyHostToDevice));
  if (cb) HIPCHK(hipMemcpy(d + vb + wb, crcs.data(), cb, hipMemcpyHostToDevice));
  if (cb) HIPCHK(hipMemcpy(d + vb + wb + cb, pos.data(), cb, hipMemcpyHostToDevice));
  if (pb) HIPCHK(hipMemcpy(d + vb + wb + 2 * cb, chunks.data(), pb, hipMemcpyHostToDevice));
  uint32_t* status = (uint32_t*)(d + vb - 16);
  HIPCHK(hipMemsetAsync(status, 0, 4, e->stream));
  HIPCHK(launch_scatter_replica(admin(e), rid, d, (const uint64_t*)(d + vb), (const uint32_t*)(d + vb + wb),
                                (const uint32_t*)(d + vb + wb + cb), pb ? d + vb + wb + 2 * cb : nullptr, nent,
                                (uint32_t)nch, status, e->stream));
  {  // no snapshot event, pending or ready read until it steps (device rows are indexed by q = s·G + g)
    const uint64_t q = (uint64_t)(rid % e->c.replicas) * e->c.groups + rid / e->c.replicas;
    HIPCHK(hipMemsetAsync(e->feed + q, 0, 8, e->stream));  // nothing to apply or persist either
    HIPCHK(hipMemsetAsync(e->rdst + (uint64_t)RQ_N * e->nrep + q, 0, 8, e->stream));
    HIPCHK(hipMemsetAsync(e->rdst + (uint64_t)RD_TICK * e->nrep + q, 0, 8, e->stream));
  }
  uint32_t st = 0;
  HIPCHK(hipMemcpyAsync(&st, status, 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (st) return fail(RG_ENOMEM, "rg_import_replica: the payload page pool is empty");
  return RG_OK;
}

int rg_deliver(rg_engine* e, uint32_t rid_src, const rg_msg_view* m) {
  if (!e || !m || rid_src >= e->nrep) return fail(RG_EINVAL, "rg_deliver args");
  if (int jrc = join(e)) return jrc;
  const uint32_t R = e->c.replicas;
  if (m->to < 1 || m->to > R) return fail(RG_EINVAL, "rg_deliver: bad destination");
  rg_msg_view h = *m;
  if (h.from == 0) h.from = (uint8_t)(rid_src % R + 1);
  if (h.type == RG_MSG_REPLICATE && h.nent) {
    if (h.nent > e->c.max_entries_per_msg) return fail(RG_EINVAL, "rg_deliver: too many entries");
    rg_replica_view v;
    int rc = rg_read_replicas(e, rid_src, 1, &v);
    if (rc) return rc;
    if (h.log_index < v.marker || h.log_index + h.nent > v.last)
      return fail(RG_EINVAL, "rg_deliver: entries not in sender log");
  }
  int rc = stage_reserve(e, 128);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipMemcpy(e->stage, &h, sizeof h, hipMemcpyHostToDevice));
  HIPCHK(launch_deliver(admin(e), rid_src, e->stage, (uint32_t*)(e->stage + 64), e->stream));
  uint32_t status = 0;
  HIPCHK(hipMemcpyAsync(&status, e->stage + 64, 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (status) return fail(RG_EFULL, "rg_deliver: outbox slot full");
  return RG_OK;
}

int rg_leader(rg_engine* e, uint32_t group, uint64_t* leader_id, uint64_t* term, int* valid) {
  const uint32_t N = e ? e->pl.N : 1;
  const uint64_t g0 = e ? (uint64_t)N * e->pl.col_base : 0;
  if (!e || group < g0 || (uint64_t)group >= g0 + (uint64_t)e->c.groups * N) return fail(RG_EINVAL, "rg_leader: bad group");
  const uint32_t R = e->c.replicas, j = group / N - e->pl.col_base;
  std::vector<rg_replica_view> v;
  for (uint32_t s = 0; s < R; ++s) {
    if (pl_rank_of(e->pl, group, s) != e->pl.rank) continue;  // replica hosted elsewhere
    rg_replica_view x;
    int rc = rg_read_replicas(e, j * R + s, 1, &x);
    if (rc) return rc;
    v.push_back(x);
  }
  if (v.empty()) return fail(RG_EINVAL, "rg_leader: no replica of this group on this rank");
  uint64_t bt = 0, bl = 0;
  for (auto& r : v) bt = std::max(bt, r.term);
  for (auto& r : v)
    if (r.role == RG_LEADER && r.term == bt) bl = r.leader;  // a leader valid at the highest local term
  if (!bl)
    for (auto& r : v)
      if (r.term == bt && r.leader) bl = r.leader;  // else the leader the replica follows
  if (leader_id) *leader_id = bl;
  if (term) *term = bt;
  if (valid) *valid = bl != 0;
  return RG_OK;
}

// device staging for the copy-back paths (grown on demand)
static int astage_reserve(rg_engine* e, uint64_t bytes) {
  if (bytes <= e->astage_bytes) return RG_OK;
  if (e->astage) {
    (void)hipFree(e->astage);
    e->allocs.erase(std::remove(e->allocs.begin(), e->allocs.end(), (void*)e->astage), e->allocs.end());
    e->bytes -= e->astage_bytes;
    e->astage = nullptr;
    e->astage_bytes = 0;
  }
  const uint64_t nb = std::max<uint64_t>(bytes * 5 / 4, 1 << 20);
  RGCHK(dalloc(e, &e->astage, nb));
  e->astage_bytes = nb;
  return RG_OK;
}

static PersistParams persist_params(rg_engine* e, bool full, uint32_t slot_mask) {
  const TickParams t = params(e);
  PersistParams a{};
  a.G = t.G; a.R = t.R; a.nrep = t.nrep; a.L = t.L; a.P = t.P; a.pl = e->pl;
  a.full = (full || e->t == 0) ? 1u : 0u;  // before the first tick there is no previous state
  a.slot_mask = slot_mask;
  a.s64 = t.s64; a.s32 = t.s32; a.feed = e->feed;
  a.tr = e->tr; a.info = e->info; a.pool = e->pool; a.pt = e->pt; a.PTS = e->PTS; a.zi = e->crc_tab + CRC_ZI_OFF;
  a.scnt = e->pscnt; a.ecnt = e->pecnt; a.ccnt = e->pccnt; a.tcnt = e->ptcnt;
  a.soff = e->psoff; a.eoff = e->peoff; a.coff = e->pcoff; a.toff = e->ptoff;
  a.bsum = e->absum;
  return a;
}
// the persist staging layout: [states][entries][terms][payload], each 16-B aligned (tot: states,
// entries, chunks, terms)
struct PersistLayout {
  uint64_t states, entries, terms, pay, total;
};
static PersistLayout persist_layout(const uint64_t* tot) {
  PersistLayout l;
  l.states = 0;
  l.entries = a16(tot[0] * sizeof(rg_persist_state));
  l.terms = l.entries + a16(tot[1] * sizeof(rg_persist_entry));
  l.pay = l.terms + a16(tot[3] * sizeof(rg_persist_term));
  l.total = tot[0] ? l.pay + tot[2] * 16 : 0;
  return l;
}
static void persist_out(PersistParams& a, uint8_t* d, const PersistLayout& l) {
  a.out_state = d + l.states;
  a.out_ent = d + l.entries;
  a.out_term = d + l.terms;
  a.out_pay = d + l.pay;
}
static void persist_batch(rg_persist_batch* out, const uint8_t* h, const uint64_t* tot, const PersistLayout& l) {
  out->states = (const rg_persist_state*)(h + l.states);
  out->n_states = tot[0];
  out->entries = (const rg_persist_entry*)(h + l.entries);
  out->n_entries = tot[1];
  out->terms = (const rg_persist_term*)(h + l.terms);
  out->n_terms = tot[3];
  out->payload = h + l.pay;
  out->payload_bytes = tot[2] * 16;
}

int rg_persist_collect(rg_engine* e, int full, rg_persist_batch* out) {
  if (!e || !out) return fail(RG_EINVAL, "rg_persist_collect args");
  if (int jrc = join(e)) return jrc;
  *out = rg_persist_batch{};
  PersistParams a = persist_params(e, full != 0, ~0u);  // every replica this engine hosts
  LAUNCH(launch_persist_count(a, (uint64_t*)e->d_sum, e->stream), e->stream, "persist count");
  uint64_t tot[4] = {0, 0, 0, 0};
  HIPCHK(hipMemcpyAsync(tot, e->d_sum, 32, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (tot[0] == 0) return RG_OK;
  const PersistLayout l = persist_layout(tot);
  RGCHK(astage_reserve(e, l.total));
  if (l.total > e->pc_hcap) {
    if (e->pc_host) (void)hipHostFree(e->pc_host);
    e->pc_host = nullptr;
    e->pc_hcap = 0;
    const uint64_t nb = std::max<uint64_t>(l.total * 5 / 4, 1 << 20);
    if (hipHostMalloc((void**)&e->pc_host, nb, 0) != hipSuccess) return fail(RG_ENOMEM, "hipHostMalloc (persist)");
    e->pc_hcap = nb;
  }
  persist_out(a, e->astage, l);
  LAUNCH(launch_persist_gather(a, e->stream), e->stream, "persist gather");
  HIPCHK(hipMemcpyAsync(e->pc_host, e->astage, l.total, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  persist_batch(out, e->pc_host, tot, l);
  return RG_OK;
}

static ApplyParams apply_params(rg_engine* e, uint32_t slot_mask) {
  const TickParams t = params(e);
  ApplyParams a{};
  a.G = t.G; a.R = t.R; a.nrep = t.nrep; a.L = t.L; a.P = t.P; a.slot_mask = slot_mask; a.pl = e->pl;
  a.s64 = t.s64; a.feed = e->feed; a.tr = e->tr; a.info = e->info;
  a.pool = e->pool; a.pt = e->pt; a.PTS = e->PTS;
  a.zi = e->crc_tab + CRC_ZI_OFF;
  a.cnt = e->acnt; a.ccnt = e->accnt; a.off = e->aoff; a.coff = e->acoff; a.bsum = e->absum;
  a.rcnt = e->arcnt; a.roff = e->aroff;
  return a;
}

// the apply staging layout: [runs][cmds][payload], each 16-B aligned (tot: entries, chunks, runs)
struct ApplyLayout {
  uint64_t runs, cmds, pay, total;
};
static ApplyLayout apply_layout(const uint64_t* tot) {
  ApplyLayout l;
  l.runs = 0;
  l.cmds = a16(tot[2] * sizeof(rg_apply_run));
  l.pay = l.cmds + a16(tot[0] * sizeof(rg_apply_cmd));
  l.total = l.pay + tot[1] * 16;
  return l;
}
static void apply_batch(rg_apply_batch* out, const uint8_t* h, const uint64_t* tot, const ApplyLayout& l) {
  out->runs = (const rg_apply_run*)(h + l.runs);
  out->n_runs = tot[2];
  out->cmds = (const rg_apply_cmd*)(h + l.cmds);
  out->n_entries = tot[0];
  out->payload = h + l.pay;
  out->payload_bytes = tot[1] * 16;
}

int rg_apply_committed(rg_engine* e, uint32_t slot_mask, rg_apply_batch* out) {
  if (!e || !out) return fail(RG_EINVAL, "rg_apply_committed args");
  if (int jrc = join(e)) return jrc;
  *out = rg_apply_batch{};
  ApplyParams a = apply_params(e, slot_mask);
  LAUNCH(launch_apply_count(a, (uint64_t*)e->d_sum, e->stream), e->stream, "apply count");
  uint64_t tot[3] = {0, 0, 0};
  HIPCHK(hipMemcpyAsync(tot, e->d_sum, 24, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (tot[0] == 0) return RG_OK;
  const ApplyLayout l = apply_layout(tot);
  RGCHK(astage_reserve(e, l.total));
  if (l.total > e->ac_hcap) {
    if (e->ac_host) (void)hipHostFree(e->ac_host);
    e->ac_host = nullptr;
    e->ac_hcap = 0;
    const uint64_t nb = std::max<uint64_t>(l.total * 5 / 4, 1 << 20);
    if (hipHostMalloc((void**)&e->ac_host, nb, 0) != hipSuccess) return fail(RG_ENOMEM, "hipHostMalloc (apply)");
    e->ac_hcap = nb;
  }
  a.out_run = e->astage + l.runs;
  a.out_cmd = e->astage + l.cmds;
  a.out_pay = e->astage + l.pay;
  LAUNCH(launch_apply_gather(a, tot[2], e->stream), e->stream, "apply gather");
  HIPCHK(hipMemcpyAsync(e->ac_host, e->astage, l.total, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  apply_batch(out, e->ac_host, tot, l);
  return RG_OK;
}

// Asynchronous copy-back: the gather runs on the engine stream right after the tick (the next tick
// may reuse the window's log slots and release its pages) into device staging; then a copy kernel
// with a handful of workgroups on the copy stream moves the staging into host-mapped pinned memory
// over PCIe. The runtime's own D2H path (blit kernels over the whole chip, measured r02) slowed the
// next ticks' kernels beside it; a few workgroups are enough to keep PCIe busy.
int rg_apply_async(rg_engine* e, uint32_t slot_mask, int buf) {
  if (!e || buf < 0 || buf > 1) return fail(RG_EINVAL, "rg_apply_async args");
  if (int jrc = join(e)) return jrc;
  ApplyParams a = apply_params(e, slot_mask);
  LAUNCH(launch_apply_count(a, (uint64_t*)e->d_sum, e->stream), e->stream, "apply count");
  uint64_t tot[3] = {0, 0, 0};
  HIPCHK(hipMemcpyAsync(tot, e->d_sum, 24, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  const ApplyLayout l = apply_layout(tot);
  const uint64_t total = tot[0], need = l.total;
  if (need > e->a_dcap[buf] || need > e->a_hcap[buf]) {  // grow: the buffer's last copy must be done
    HIPCHK(hipEventSynchronize(e->a_copy[buf]));
    if (e->sdma) sdma_wait(e->sdma, buf);
    const uint64_t nb = std::max<uint64_t>(need * 5 / 4, 1 << 20);
    if (need > e->a_dcap[buf]) {
      if (e->a_dev[buf]) {
        (void)hipFree(e->a_dev[buf]);
        e->allocs.erase(std::remove(e->allocs.begin(), e->allocs.end(), (void*)e->a_dev[buf]), e->allocs.end());
        e->bytes -= e->a_dcap[buf];
        e->a_dev[buf] = nullptr;
      }
      e->a_dcap[buf] = 0;
      RGCHK(dalloc(e, &e->a_dev[buf], nb));
      e->a_dcap[buf] = nb;
    }
    if (need > e->a_hcap[buf]) {
      if (e->a_host[buf]) (void)hipHostFree(e->a_host[buf]);
      e->a_host[buf] = nullptr;
      e->a_hcap[buf] = 0;
      if (hipHostMalloc((void**)&e->a_host[buf], nb, hipHostMallocMapped) != hipSuccess)
        return fail(RG_ENOMEM, "hipHostMalloc (apply)");
      e->a_hcap[buf] = nb;
    }
  }
  const bool prev = e->a_used[buf];
  e->a_n[buf] = total;
  for (int k = 0; k < 3; ++k) e->a_tot[buf][k] = tot[k];
  e->a_used[buf] = true;
  if (total) {
    if (prev && e->sdma) sdma_wait(e->sdma, buf);  // its last copy has read the staging
    else if (prev) HIPCHK(hipStreamWaitEvent(e->stream, e->a_copy[buf], 0));
    a.out_run = e->a_dev[buf] + l.runs;
    a.out_cmd = e->a_dev[buf] + l.cmds;
    a.out_pay = e->a_dev[buf] + l.pay;
    LAUNCH(launch_apply_gather(a, tot[2], e->stream), e->stream, "apply gather");
  }
  HIPCHK(hipEventRecord(e->a_gath[buf], e->stream));
  if (e->sdma) {  // the DMA engine takes the batch once the gather is done (no shader code on the copy)
    if (total) {
      HIPCHK(hipEventSynchronize(e->a_gath[buf]));
      if (sdma_copy(e->sdma, buf, e->a_host[buf], e->a_dev[buf], need) != 0)
        return fail(RG_EHIP, "rg_apply_async: hsa_amd_memory_async_copy failed");
    }
    return RG_OK;
  }
  HIPCHK(hipStreamWaitEvent(e->copy, e->a_gath[buf], 0));
  if (total) {
    if (e->copy_kernel) {
      void* hdev = nullptr;
      HIPCHK(hipHostGetDevicePointer(&hdev, e->a_host[buf], 0));
      LAUNCH(launch_copy_to_host(e->a_dev[buf], hdev, need, e->copy), e->copy, "copy to host");
    } else {
      HIPCHK(hipMemcpyAsync(e->a_host[buf], e->a_dev[buf], need, hipMemcpyDeviceToHost, e->copy));
    }
  }
  HIPCHK(hipEventRecord(e->a_copy[buf], e->copy));
  return RG_OK;
}

int rg_apply_wait(rg_engine* e, int buf, rg_apply_batch* out) {
  if (!e || buf < 0 || buf > 1 || !out) return fail(RG_EINVAL, "rg_apply_wait args");
  if (!e->a_used[buf]) return fail(RG_EINVAL, "rg_apply_wait: no rg_apply_async into this buffer");
  if (e->sdma) sdma_wait(e->sdma, buf);
  else HIPCHK(hipEventSynchronize(e->a_copy[buf]));
  *out = rg_apply_batch{};
  if (e->a_n[buf]) apply_batch(out, e->a_host[buf], e->a_tot[buf], apply_layout(e->a_tot[buf]));
  return RG_OK;
}

int rg_pool_stats(rg_engine* e, uint64_t* total_pages, uint64_t* free_pages, int* failed) {
  if (!e) return fail(RG_EINVAL, "rg_pool_stats args");
  if (int jrc = join(e)) return jrc;
  PoolCtl c{};
  HIPCHK(hipMemcpyAsync(&c, e->poolctl, sizeof c, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (total_pages) *total_pages = e->npages;
  if (free_pages) *free_pages = c.tail >= c.head ? c.tail - c.head : 0;
  if (failed) *failed = c.fail ? 1 : 0;
  return RG_OK;
}

int rg_snapshot_events(rg_engine* e, uint32_t slot_mask, rg_snapshot_event* events, uint64_t cap, uint64_t* n) {
  if (!e || !n) return fail(RG_EINVAL, "rg_snapshot_events args");
  if (int jrc = join(e)) return jrc;
  const TickParams t = params(e);
  SnapParams a{};
  a.G = t.G; a.R = t.R; a.nrep = t.nrep; a.slot_mask = slot_mask; a.pl = e->pl;
  a.s64 = t.s64; a.feed = e->feed;
  a.cnt = e->acnt; a.off = e->aoff; a.bsum = e->absum;
  LAUNCH(launch_snap_count(a, (uint64_t*)e->d_sum, e->stream), e->stream, "snapshot count");
  uint64_t total = 0;
  HIPCHK(hipMemcpyAsync(&total, e->d_sum, 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  *n = total;
  if (total == 0) return RG_OK;
  if (total > cap) return fail(RG_EFULL, "rg_snapshot_events: " + std::to_string(total) + " events > cap");
  if (!events) return fail(RG_EINVAL, "rg_snapshot_events: null output");
  const uint64_t rb = total * sizeof(rg_snapshot_event);
  RGCHK(astage_reserve(e, rb));
  a.out = e->astage;
  LAUNCH(launch_snap_gather(a, e->stream), e->stream, "snapshot gather");
  HIPCHK(hipMemcpyAsync(events, a.out, rb, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return RG_OK;
}

#ifdef RG_CTL_PROFILE
// measurement builds only (not in include/raftgpu.h): the last control launch's phase stamps
extern "C" int rg_debug_ctl_profile(rg_engine* e, uint32_t* out) {
  if (!e || !out) return fail(RG_EINVAL, "rg_debug_ctl_profile args");
  if (int jrc = join(e)) return jrc;
  HIPCHK(hipMemcpy(out, e->prof, (uint64_t)e->nrep * 12 * 4, hipMemcpyDeviceToHost));
  return RG_OK;
}
#endif

// measurement / tests (not in include/raftgpu.h): replicas of the last tick whose step left the control
// fast path and ran in the full kernel (0 in the -DRG_AB_CTL_FULL build)
extern "C" int rg_debug_ctl_slow(rg_engine* e, uint32_t* n) {
  if (!e || !n) return fail(RG_EINVAL, "rg_debug_ctl_slow args");
  if (int jrc = join(e)) return jrc;
  *n = 0;
  if (!e->ctl_fast || e->t == 0) return RG_OK;
  HIPCHK(hipMemcpyAsync(n, e->slow + ((e->t - 1) & 1), 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return RG_OK;
}

// measurement / tests (not in include/raftgpu.h): parameter-block copies issued so far (launch_control_slot:
// one per TP_CHUNK ticks in the steady state, one more per tick whose block differs from the speculated one)
extern "C" int rg_debug_param_copies(rg_engine* e, uint64_t* n) {
  if (!e || !n) return fail(RG_EINVAL, "rg_debug_param_copies args");
  *n = e->tp_copies;
  return RG_OK;
}

// tests only (not in include/raftgpu.h): the next n control launches get a parameter block whose
// checksum does not match (the control kernel must skip the tick, the pool and payload stages must
// not act on its stale rows, and the next rg_sync must report RG_EINVARIANT)
extern "C" int rg_debug_corrupt_params(rg_engine* e, uint32_t n) {
  if (!e) return fail(RG_EINVAL, "null engine");
  e->tp_corrupt = n;
  return RG_OK;
}

// tests only (not in include/raftgpu.h): where this process's kernel arguments live.
// *is_device = 1 device memory, 0 host memory, -1 unknown (the runtime does not track the address)
extern "C" int rg_debug_kernarg_placement(int32_t device, uint64_t* addr, int32_t* is_device) {
  if (!addr || !is_device) return fail(RG_EINVAL, "rg_debug_kernarg_placement args");
  HIPCHK(hipSetDevice(device));
  uint64_t* d = nullptr;
  HIPCHK(hipMalloc((void**)&d, 16));
  uint64_t h[2] = {0, 0};
  hipError_t r = launch_kernarg_probe(d, 0x5EEDull, nullptr);
  if (r == hipSuccess) r = hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (r != hipSuccess) return fail(RG_EHIP, std::string("kernarg probe: ") + hipGetErrorString(r));
  if (h[1] != 0x5EEDull) return fail(RG_EHIP, "kernarg probe: bad tag");
  *addr = h[0];
  hipPointerAttribute_t at{};
  *is_device = -1;
  if (hipPointerGetAttributes(&at, (void*)(uintptr_t)h[0]) == hipSuccess)
    *is_device = at.type == hipMemoryTypeDevice ? 1 : at.type == hipMemoryTypeHost ? 0 : -1;
  (void)hipGetLastError();
  return RG_OK;
}

int rg_config_change(rg_engine* e, uint64_t group, uint32_t slot, uint32_t op, uint32_t target) {
  if (!e) return fail(RG_EINVAL, "rg_config_change args");
  const uint32_t N = e->pl.N, R = e->c.replicas;
  const uint64_t g0 = (uint64_t)N * e->pl.col_base, gn = (uint64_t)N * e->c.groups;
  if (group < g0 || group >= g0 + gn || slot >= R || target >= R || (op != RG_CC_ADD && op != RG_CC_REMOVE))
    return fail(RG_EINVAL, "rg_config_change: bad shard, slot, target or op");
  if (pl_rank_of(e->pl, group, slot) != e->pl.rank)
    return fail(RG_EINVAL, "rg_config_change: replica hosted by another rank");
  if (e->cc_reset_pending) {  // the last upload has completed: clear what it carried
    HIPCHK(hipEventSynchronize(e->cc_ev));
    for (uint64_t i : e->cc_touched) e->h_cc[i] = 0;
    e->cc_touched.clear();
    e->cc_reset_pending = false;
  }
  const uint64_t gi = group - g0;
  if (e->h_cc[gi]) return fail(RG_EFULL, "rg_config_change: a change is already staged for this shard");
  e->h_cc[gi] = (uint16_t)(slot | ((op << 4 | (target + 1u)) << 8));
  e->cc_touched.push_back(gi);
  e->cc_staged = true;
  return RG_OK;
}

int rg_read_index(rg_engine* e, const rg_read_request* reqs, size_t n) {
  if (!e || (n && !reqs)) return fail(RG_EINVAL, "rg_read_index args");
  if (e->rd_reset_pending) {  // the last upload has completed: clear what it carried
    HIPCHK(hipEventSynchronize(e->rd_ev));
    for (uint64_t i : e->rd_touched) e->h_rd[i] = 0;
    e->rd_touched.clear();
    e->rd_reset_pending = false;
  }
  const uint32_t N = e->pl.N, R = e->c.replicas;
  const uint64_t g0 = (uint64_t)N * e->pl.col_base, gn = (uint64_t)N * e->c.groups;
  for (size_t i = 0; i < n; ++i) {
    const rg_read_request& q = reqs[i];
    if (q.group < g0 || q.group >= g0 + gn || q.slot >= R || q.ctx == 0)
      return fail(RG_EINVAL, "rg_read_index: request " + std::to_string(i) + ": bad shard, slot or ctx 0");
    if (pl_rank_of(e->pl, q.group, q.slot) != e->pl.rank)
      return fail(RG_EINVAL, "rg_read_index: request " + std::to_string(i) + ": replica hosted by another rank");
  }
  for (size_t i = 0; i < n; ++i) {
    const uint64_t at = (reqs[i].group - g0) * R + reqs[i].slot;
    if (!e->h_rd[at]) e->rd_touched.push_back(at);
    e->h_rd[at] = reqs[i].ctx;
  }
  if (n) e->rd_staged = true;
  return RG_OK;
}

int rg_read_index_results(rg_engine* e, uint32_t slot_mask, rg_read_ready* out, uint64_t cap, uint64_t* n) {
  if (!e || !n) return fail(RG_EINVAL, "rg_read_index_results args");
  if (int jrc = join(e)) return jrc;
  const TickParams t = params(e);
  SnapParams a{};
  a.G = t.G; a.R = t.R; a.nrep = t.nrep; a.slot_mask = slot_mask; a.pl = e->pl;
  a.s64 = t.s64; a.rdst = e->rdst; a.tick = e->t;
  a.cnt = e->acnt; a.off = e->aoff; a.bsum = e->absum;
  LAUNCH(launch_read_count(a, (uint64_t*)e->d_sum, e->stream), e->stream, "read count");
  uint64_t total = 0;
  HIPCHK(hipMemcpyAsync(&total, e->d_sum, 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  *n = total;
  if (total == 0) return RG_OK;
  if (total > cap) return fail(RG_EFULL, "rg_read_index_results: " + std::to_string(total) + " > cap");
  if (!out) return fail(RG_EINVAL, "rg_read_index_results: null output");
  const uint64_t rb = total * sizeof(rg_read_ready);
  RGCHK(astage_reserve(e, rb));
  a.out = e->astage;
  LAUNCH(launch_read_gather(a, e->stream), e->stream, "read gather");
  HIPCHK(hipMemcpyAsync(out, a.out, rb, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return RG_OK;
}

// rg_get_update: every section's count kernels first (their totals side by side in d_sum), one
// synchronisation, every section's gather into one device staging area, one D2H copy, one
// synchronisation — instead of a count, sync, gather, copy and sync per section
int rg_get_update(rg_engine* e, uint32_t slot_mask, uint32_t flags, rg_update* out) {
  if (!e || !out || (flags & ~(RG_UPDATE_ALL | RG_UPDATE_FULL_STATE | RG_UPDATE_COMMITTED_CMDS)))
    return fail(RG_EINVAL, "rg_get_update args");
  // the committed section by reference: with the persist section in the same hand-off every committed
  // entry's Cmd has crossed once already (this or an earlier persist section of the same replicas), so
  // only its run, length and CRC cross again (the hand-off shipped every Cmd twice)
  const bool by_ref = (flags & RG_UPDATE_PERSIST) && (flags & RG_UPDATE_COMMITTED) && !(flags & RG_UPDATE_COMMITTED_CMDS);
  if (int jrc = join(e)) return jrc;
  *out = rg_update{};
  out->tick = e->t;
  out->slot_mask = slot_mask;
  out->flags = flags;
  const TickParams t = params(e);
  // [0..3] persist (states, entries, chunks, terms), [4..6] committed (entries, chunks, runs),
  // [7] snapshots, [8] reads
  uint64_t* sum = (uint64_t*)e->d_sum;
  // a node persists its own replicas only (4.3 GB of others' entries)
  PersistParams pa = persist_params(e, (flags & RG_UPDATE_FULL_STATE) != 0, slot_mask);
  ApplyParams aa = apply_params(e, slot_mask);
  SnapParams sa{};
  sa.G = t.G; sa.R = t.R; sa.nrep = t.nrep; sa.slot_mask = slot_mask; sa.pl = e->pl;
  sa.s64 = t.s64; sa.feed = e->feed; sa.rdst = e->rdst; sa.tick = e->t;
  sa.cnt = e->uscnt; sa.off = e->usoff; sa.bsum = e->absum;
  SnapParams ra = sa;
  ra.cnt = e->urcnt; ra.off = e->uroff;
  HIPCHK(hipMemsetAsync(sum, 0, D_SUM_BYTES, e->stream));
  if (flags & RG_UPDATE_PERSIST) LAUNCH(launch_persist_count(pa, sum, e->stream), e->stream, "persist count");
  if (flags & RG_UPDATE_COMMITTED) LAUNCH(launch_apply_count(aa, sum + 4, e->stream), e->stream, "apply count");
  if (flags & RG_UPDATE_SNAPSHOTS) LAUNCH(launch_snap_count(sa, sum + 7, e->stream), e->stream, "snapshot count");
  if (flags & RG_UPDATE_READS) LAUNCH(launch_read_count(ra, sum + 8, e->stream), e->stream, "read count");
  uint64_t tot[D_SUM_BYTES / 8] = {};
  HIPCHK(hipMemcpyAsync(tot, sum, D_SUM_BYTES, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  // one staging layout for every section, each 16-B aligned
  const PersistLayout pl = persist_layout(tot);
  const uint64_t ctot[3] = {tot[4], by_ref ? 0 : tot[5], tot[6]};
  const ApplyLayout al = apply_layout(ctot);  // committed: entries, chunks (none by reference), runs
  const uint64_t snb = a16(tot[7] * sizeof(rg_snapshot_event)), rdb = a16(tot[8] * sizeof(rg_read_ready));
  const uint64_t o_c = pl.total, o_s = o_c + al.total, o_r = o_s + snb, total = o_r + rdb;
  if (total == 0) return RG_OK;
  RGCHK(astage_reserve(e, total));
  if (total > e->u_hcap) {
    if (e->u_host) (void)hipHostFree(e->u_host);
    e->u_host = nullptr;
    e->u_hcap = 0;
    const uint64_t nb = std::max<uint64_t>(total * 5 / 4, 1 << 20);
    if (hipHostMalloc((void**)&e->u_host, nb, 0) != hipSuccess) return fail(RG_ENOMEM, "hipHostMalloc (update)");
    e->u_hcap = nb;
  }
  uint8_t* d = e->astage;
  if (tot[0]) {
    persist_out(pa, d, pl);
    LAUNCH(launch_persist_gather(pa, e->stream), e->stream, "persist gather");
  }
  if (tot[4]) {
    aa.out_run = d + o_c + al.runs;
    aa.out_cmd = d + o_c + al.cmds;
    aa.out_pay = by_ref ? nullptr : d + o_c + al.pay;
    LAUNCH(launch_apply_gather(aa, tot[6], e->stream), e->stream, "apply gather");
  }
  if (tot[7]) {
    sa.out = d + o_s;
    LAUNCH(launch_snap_gather(sa, e->stream), e->stream, "snapshot gather");
  }
  if (tot[8]) {
    ra.out = d + o_r;
    LAUNCH(launch_read_gather(ra, e->stream), e->stream, "read gather");
  }
  HIPCHK(hipMemcpyAsync(e->u_host, d, total, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  uint8_t* h = e->u_host;
  if (tot[0]) persist_batch(&out->persist, h, tot, pl);
  out->committed = rg_apply_batch{};
  if (tot[4]) {
    apply_batch(&out->committed, h + o_c, ctot, al);
    if (by_ref) out->committed.payload = nullptr;  // runs' off: where each Cmd would sit, packed
  }
  out->snapshots = (const rg_snapshot_event*)(h + o_s);
  out->n_snapshots = tot[7];
  out->reads = (const rg_read_ready*)(h + o_r);
  out->n_reads = tot[8];
  return RG_OK;
}

int rg_digest(rg_engine* e, uint64_t* out) {
  if (!e || !out) return fail(RG_EINVAL, "rg_digest args");
  if (int jrc = join(e)) return jrc;
  HIPCHK(hipMemsetAsync(e->d_sum, 0, 16, e->stream));
  LAUNCH(launch_digest(admin(e), e->d_sum, e->stream), e->stream, "digest");
  HIPCHK(hipMemcpyAsync(out, e->d_sum, 16, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return RG_OK;
}

int rg_commit_update(rg_engine* e, const rg_update* u, uint32_t flags) {
  if (!e || !u || (flags & ~RG_COMMIT_APPLIED)) return fail(RG_EINVAL, "rg_commit_update args");
  if (u->tick != e->t) return fail(RG_EINVAL, "rg_commit_update: the update is not of the last tick");
  if (flags & RG_COMMIT_APPLIED) {
    if (int jrc = join(e)) return jrc;
    LAUNCH(launch_applied_all(admin(e), u->slot_mask, e->stream), e->stream, "applied all");
  }
  return RG_OK;
}

int rg_notify_applied(rg_engine* e, const uint32_t* rids, const uint64_t* index, size_t n) {
  if (!e || (n && (!rids || !index))) return fail(RG_EINVAL, "rg_notify_applied args");
  if (n == 0) return RG_OK;
  if (n > 0x7FFFFFFFull) return fail(RG_EINVAL, "rg_notify_applied: too many");
  if (int jrc = join(e)) return jrc;
  const uint64_t rb = (n * 4 + 15) & ~15ull, ib = n * 8;
  RGCHK(stage_reserve(e, rb + ib + 16));
  uint8_t* d = e->stage;
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipMemcpy(d, rids, n * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d + rb, index, ib, hipMemcpyHostToDevice));
  uint32_t* bad = (uint32_t*)(d + rb + ib);
  HIPCHK(hipMemsetAsync(bad, 0, 4, e->stream));
  HIPCHK(launch_notify_applied(admin(e), (const uint32_t*)d, (const uint64_t*)(d + rb), (uint32_t)n, 0, bad, e->stream));
  uint32_t nbad = 0;
  HIPCHK(hipMemcpyAsync(&nbad, bad, 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (nbad) return fail(RG_EINVAL, "rg_notify_applied: " + std::to_string(nbad) + " replica(s) bad or past processed");
  HIPCHK(launch_notify_applied(admin(e), (const uint32_t*)d, (const uint64_t*)(d + rb), (uint32_t)n, 1, bad, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return RG_OK;
}

int rg_compact(rg_engine* e, uint64_t group, uint64_t index, uint32_t* compacted) {
  if (!e) return fail(RG_EINVAL, "rg_compact args");
  const uint32_t N = e->pl.N;
  const uint64_t g0 = (uint64_t)N * e->pl.col_base, gn = (uint64_t)N * e->c.groups;
  if (group < g0 || group >= g0 + gn) return fail(RG_EINVAL, "rg_compact: shard outside this engine");
  if (int jrc = join(e)) return jrc;
  HIPCHK(hipSetDevice(e->c.device));
  uint32_t* d = (uint32_t*)e->d_sum;
  HIPCHK(hipMemsetAsync(d, 0, 4, e->stream));
  HIPCHK(launch_compact(admin(e), group, index, d, e->stream));
  uint32_t n = 0;
  HIPCHK(hipMemcpyAsync(&n, d, 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (compacted) *compacted = n;
  return RG_OK;
}

int rg_global_id(rg_engine* e, uint32_t rid, uint64_t* group, uint64_t* global_rid) {
  if (!e || rid >= e->nrep) return fail(RG_EINVAL, "rg_global_id: bad replica");
  const uint32_t R = e->c.replicas, j = rid / R, s = rid % R;
  const uint64_t gg = pl_group(e->pl, s, j);
  if (group) *group = gg;
  if (global_rid) *global_rid = gg * R + s;
  return RG_OK;
}

int rg_wire_plan(rg_engine* e, uint64_t* send_bytes) {
  if (!e || !send_bytes) return fail(RG_EINVAL, "rg_wire_plan args");
  const uint32_t N = e->pl.N;
  if (!e->wire) {
    for (uint32_t r = 0; r < N; ++r) send_bytes[r] = 0;
    return RG_OK;
  }
  if (int jrc = join(e)) return jrc;
  HIPCHK(hipSetDevice(e->c.device));
  LAUNCH(launch_wire_plan(wire_params(e), e->bounds, e->stream), e->stream, "wire plan");
  HIPCHK(hipMemcpyAsync(e->h_bounds, e->bounds, (N + 1) * 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  for (uint32_t r = 0; r < N; ++r) {
    const uint64_t units = e->h_ubeg[r + 1] - e->h_ubeg[r], data = (e->h_bounds[r + 1] - e->h_bounds[r]) * 16;
    e->send_bytes[r] = units ? wire_region_min(units) + ((data + 255) & ~255ull) : 0;
    send_bytes[r] = e->send_bytes[r];
  }
  e->planned = true;
  e->fixed = false;
  return RG_OK;
}

// Fixed-capacity regions. A transfer moves a link's whole capacity, and no rank may
// ask another what it needs, so each end of a link (a → b) computes the capacity by the same rule from
// the same numbers: the bytes the link's region asked for in each exchange (the sender from its plan,
// the receiver from the region's header), two exchanges late, so neither waits on the current tick.
// * Start: the worst case (K messages of E entries of max_cmd_bytes per unit) when it is at most
//   64 MiB — such a link never shrinks below it, so it never drops — else the most the units can need
//   in a steady tick, a full Replicate plus one more header per unit (at least 64 MiB).
// * Follow: 1/16 + 64 KiB above the largest need of the last WIRE_WIN exchanges; a need past the
//   capacity (its units were dropped: lost in transit, counted) takes it to 1.5 × that need at once;
//   a capacity above the target shrinks by at most 1/8 per exchange (bring-up's small needs do not
//   undersize it before the load arrives, and a steady load settles 6 % above its need).
// * Floor: a large link never shrinks below min(its start, 64 MiB) (with the region's bare
//   minimum as the floor, ~30 quiet exchanges took it to a few KiB and the next burst was dropped whole
//   for two exchanges); a link whose worst case fits keeps its start, as before.
// RAFTGPU_WIRE_CAP0 (tests) caps the start, to exercise the drop-and-grow path.
static constexpr uint64_t WIRE_CAP_MAX = 4ull << 30;
static constexpr uint32_t WIRE_WIN = 8;  // exchanges a capacity looks back over
static constexpr uint64_t WIRE_CAP_SMALL = 64ull << 20;
static void wire_caps_init(rg_engine* e) {
  const uint32_t N = e->pl.N;
  uint64_t cap0 = ~0ull;
  if (const char* v = getenv("RAFTGPU_WIRE_CAP0")) cap0 = std::max<uint64_t>(strtoull(v, nullptr, 10), 4096);
  const uint64_t msg = 64 + (uint64_t)e->c.max_entries_per_msg * (16 + (((uint64_t)e->maxc + 15) & ~15ull));
  auto first = [&](uint64_t units, uint64_t& floor) -> uint64_t {
    floor = wire_region_min(units);
    if (!units) return 0;
    const long double worst = (long double)wire_region_min(units) + (long double)units * e->c.max_msgs_per_pair * msg;
    const long double steady = (long double)wire_region_min(units) + (long double)units * (64 + msg);
    // a link whose worst case is small keeps it (it never drops: every parity run); a larger one starts
    // at the steady bound (C3 at N = 8: ~0.4 GB per link instead of K times that)
    long double c = worst <= (long double)WIRE_CAP_SMALL ? worst
                                                          : std::max((long double)WIRE_CAP_SMALL, std::min(worst, steady));
    if (c > (long double)cap0) c = (long double)cap0;
    if (c > (long double)WIRE_CAP_MAX) c = (long double)WIRE_CAP_MAX;
    const uint64_t cap = (std::max<uint64_t>((uint64_t)c, wire_region_min(units)) + 255) & ~255ull;
    if ((long double)cap >= worst) floor = cap;  // the worst case fits: never below it, never a drop
    else floor = std::max<uint64_t>(floor, std::min<uint64_t>(cap, WIRE_CAP_SMALL));  // idle-then-burst headroom
    return cap;
  };
  e->cap_s.assign(N, 0);
  e->cap_r.assign(N, 0);
  e->cap_s0.assign(N, 0);
  e->cap_r0.assign(N, 0);
  e->win_s.assign((uint64_t)N * WIRE_WIN, 0);
  e->win_r.assign((uint64_t)N * WIRE_WIN, 0);
  for (uint32_t r = 0; r < N; ++r) {
    e->cap_s[r] = first(e->h_ubeg[r + 1] - e->h_ubeg[r], e->cap_s0[r]);
    e->cap_r[r] = first(e->h_rbeg[r + 1] - e->h_rbeg[r], e->cap_r0[r]);
  }
}
// one exchange's need into the link's window (slot k of WIRE_WIN), then the capacity rule above
static void wire_cap_adapt(uint64_t& cap, uint64_t floor, uint64_t* win, uint64_t k, uint64_t need) {
  if (!cap) return;
  win[k % WIRE_WIN] = need;
  uint64_t peak = 0;
  for (uint32_t i = 0; i < WIRE_WIN; ++i) peak = std::max(peak, win[i]);
  const uint64_t chunk = 64ull << 10;
  const uint64_t target = std::max<uint64_t>(floor, std::min<uint64_t>(WIRE_CAP_MAX, (peak + peak / 16 + 2 * chunk - 1) & ~(chunk - 1)));
  if (need > cap) cap = std::max<uint64_t>(target, std::min<uint64_t>(WIRE_CAP_MAX, (need + need / 2 + chunk - 1) & ~(chunk - 1)));
  else if (target > cap) cap = target;
  else if (target < cap) cap = std::max<uint64_t>(target, std::min<uint64_t>(cap, (cap - cap / 8 + chunk - 1) & ~(chunk - 1)));
}

int rg_wire_plan_fixed(rg_engine* e, uint64_t* send_bytes, uint64_t* recv_bytes) {
  if (!e || !send_bytes || !recv_bytes) return fail(RG_EINVAL, "rg_wire_plan_fixed args");
  const uint32_t N = e->pl.N;
  if (!e->wire) {
    for (uint32_t r = 0; r < N; ++r) send_bytes[r] = recv_bytes[r] = 0;
    return RG_OK;
  }
  if (int jrc = join(e)) return jrc;
  HIPCHK(hipSetDevice(e->c.device));
  if (e->cap_s.empty()) wire_caps_init(e);
  if (e->nfix >= 2) {
    // the needs of the exchange two before. A bounded wait: that exchange's unpack sits behind a whole
    // tick on this stream, so the host never runs more than two exchanges ahead of the device
    const uint64_t k = e->nfix - 2;
    const uint32_t sl = (uint32_t)(k % 4);
    HIPCHK(hipEventSynchronize(e->need_ev[sl]));
    const uint64_t* hn = e->h_need + (uint64_t)sl * 2 * MAX_RANKS;
    for (uint32_t r = 0; r < N; ++r)
      if (hn[MAX_RANKS + r] == ~0ull)  // unpack_kernel rejected the region header (raftgpu_wire.hip)
        return fail(RG_EINVARIANT, "rg_wire_plan_fixed: region from rank " + std::to_string(r) +
                                       " carried an impossible size: the link's capacities can no longer agree");
    for (uint32_t r = 0; r < N; ++r) {
      wire_cap_adapt(e->cap_s[r], e->cap_s0[r], &e->win_s[(uint64_t)r * WIRE_WIN], k, hn[r]);
      wire_cap_adapt(e->cap_r[r], e->cap_r0[r], &e->win_r[(uint64_t)r * WIRE_WIN], k, hn[MAX_RANKS + r]);
    }
  }
  LAUNCH(launch_wire_plan(wire_params(e), e->bounds, e->stream), e->stream, "wire plan");
  for (uint32_t r = 0; r < N; ++r) {
    e->send_bytes[r] = send_bytes[r] = e->cap_s[r];
    recv_bytes[r] = e->cap_r[r];
  }
  e->planned = true;
  e->fixed = true;
  return RG_OK;
}

int rg_wire_dropped(rg_engine* e, uint64_t* msgs) {
  if (!e || !msgs) return fail(RG_EINVAL, "rg_wire_dropped args");
  *msgs = 0;
  if (!e->wire) return RG_OK;
  if (int jrc = join(e)) return jrc;
  unsigned long long v = 0;
  HIPCHK(hipMemcpyAsync(&v, e->d_drops, 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  *msgs = v;
  return RG_OK;
}

// pack region r at base + off[r] (send_bytes[r] bytes; the regions inside cap, not overlapping)
static int wire_pack_at(rg_engine* e, void* base, const uint64_t* off, uint64_t cap, const char* who) {
  if (!e->planned) return fail(RG_EINVAL, std::string(who) + " before rg_wire_plan");
  WireParams w = wire_params(e);
  const uint32_t N = e->pl.N;
  uint64_t tot = 0;
  for (uint32_t r = 0; r < N; ++r) {
    const uint64_t n = e->send_bytes[r];
    if (!n) continue;
    if ((off[r] & 15) || off[r] > cap || n > cap - off[r])
      return fail(RG_EFULL, std::string(who) + ": region of rank " + std::to_string(r) + " outside the buffer");
    for (uint32_t o = 0; o < r; ++o)
      if (e->send_bytes[o] && off[o] < off[r] + n && off[r] < off[o] + e->send_bytes[o])
        return fail(RG_EINVAL, std::string(who) + ": regions of ranks " + std::to_string(o) + " and " +
                                   std::to_string(r) + " overlap");
    tot += n;
  }
  if (tot && !base) return fail(RG_EINVAL, std::string(who) + ": null buffer");
  for (uint32_t r = 0; r < N; ++r) {
    w.send_region[r] = off[r];
    w.send_cap[r] = e->fixed ? e->send_bytes[r] : 0;
  }
  w.send = (uint8_t*)base;
  LAUNCH(launch_wire_pack(w, e->stream), e->stream, "pack_kernel");
  e->planned = false;
  return RG_OK;
}

int rg_wire_pack(rg_engine* e, void* send_buf, uint64_t send_cap) {
  if (!e) return fail(RG_EINVAL, "null engine");
  if (!e->wire) return RG_OK;
  uint64_t off[MAX_RANKS], o = 0;
  for (uint32_t r = 0; r < e->pl.N; ++r) {
    off[r] = o;
    o += e->send_bytes[r];
  }
  if (o > send_cap) return fail(RG_EFULL, "rg_wire_pack: send buffer smaller than the planned regions");
  return wire_pack_at(e, send_buf, off, send_cap, "rg_wire_pack");
}

int rg_wire_pack_at(rg_engine* e, void* base, const uint64_t* region_off, uint64_t base_cap) {
  if (!e || !region_off) return fail(RG_EINVAL, "rg_wire_pack_at args");
  if (!e->wire) return RG_OK;
  return wire_pack_at(e, base, region_off, base_cap, "rg_wire_pack_at");
}

int rg_wire_recv(rg_engine* e, const void* recv_buf, const uint64_t* recv_bytes) {
  if (!e || !recv_bytes) return fail(RG_EINVAL, "rg_wire_recv args");
  if (!e->wire) return RG_OK;
  if (int jrc = join(e)) return jrc;
  WireParams w = wire_params(e);
  uint64_t off = 0;
  for (uint32_t r = 0; r < e->pl.N; ++r) {
    const uint64_t units = e->h_rbeg[r + 1] - e->h_rbeg[r];
    if ((units ? recv_bytes[r] < wire_region_min(units) : recv_bytes[r] != 0) || (recv_bytes[r] & 15))
      return fail(RG_EINVAL, "rg_wire_recv: region of rank " + std::to_string(r) + " has the wrong size");
    w.recv_region[r] = off;
    off += recv_bytes[r];
  }
  if (off && !recv_buf) return fail(RG_EINVAL, "rg_wire_recv: null buffer");
  w.recv = (const uint8_t*)recv_buf;
  w.recv_total = off;
  LAUNCH(launch_wire_unpack(w, e->stream), e->stream, "unpack_kernel");
  if (e->fixed) {  // this exchange's needs, for the capacity two exchanges on (no wait here)
    const uint32_t sl = (uint32_t)(e->nfix % 4);
    HIPCHK(hipMemcpyAsync(e->h_need + (uint64_t)sl * 2 * MAX_RANKS, e->d_need, 2 * MAX_RANKS * 8, hipMemcpyDeviceToHost,
                          e->stream));
    HIPCHK(hipEventRecord(e->need_ev[sl], e->stream));
    e->nfix++;
    e->fixed = false;
  }
  e->recv = (const uint8_t*)recv_buf;
  e->recv_bytes = off;
  e->wire_ready = true;
  return RG_OK;
}

int rg_sum_committed(rg_engine* e, uint64_t* out) {
  if (!e || !out) return fail(RG_EINVAL, "rg_sum_committed args");
  if (int jrc = join(e)) return jrc;
  HIPCHK(hipMemsetAsync(e->d_sum, 0, 8, e->stream));
  HIPCHK(launch_sum_committed(params(e), e->d_sum, e->stream));
  unsigned long long v = 0;
  HIPCHK(hipMemcpyAsync(&v, e->d_sum, 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  *out = v;
  return RG_OK;
}

int rg_last_tick_traffic(rg_engine* e, rg_traffic* out) {
  if (!e || !out) return fail(RG_EINVAL, "rg_last_tick_traffic args");
  if (e->t == 0) return fail(RG_EINVAL, "no tick has run");
  if (int jrc = join(e)) return jrc;
  HIPCHK(hipMemsetAsync(e->d_sum, 0, 64, e->stream));
  TickParams tp = params(e);  // the last tick's copy jobs: its appended entries
  tp.job32 = e->job32[(e->t - 1) & 1];
  tp.jcnt = e->jcnt[(e->t - 1) & 1];
  HIPCHK(launch_traffic(tp, e->d_sum, e->stream));
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
  out->bulk_bytes = (2 * P + 8) * v[3] - 4 * v[4];
  return RG_OK;
}


// One exchange between two ticks (include/raftgpu.h): plan, sizes, pack, transport, unpack.
static int xgrow(rg_engine* e, uint8_t** buf, uint64_t* cap, uint64_t need) {
  if (need <= *cap) return RG_OK;
  if (*buf) {
    HIPCHK(hipStreamSynchronize(e->stream));  // the last tick or transfer may still read it
    (void)hipFree(*buf);
    e->allocs.erase(std::remove(e->allocs.begin(), e->allocs.end(), (void*)*buf), e->allocs.end());
    e->bytes -= *cap;
    *buf = nullptr;
    *cap = 0;
  }
  const uint64_t nb = ((need + need / 4) + 4095) & ~4095ull;  // 25 % headroom against regrowth
  RGCHK(dalloc(e, buf, nb));
  *cap = nb;
  return RG_OK;
}

int rg_wire_exchange(rg_engine* e, const rg_transport* t, uint64_t* sent_bytes) {
  if (!e || !t || !t->alltoallv) return fail(RG_EINVAL, "rg_wire_exchange args");
  if (sent_bytes) *sent_bytes = 0;
  if (!e->wire) return RG_OK;
  // Sizing: fixed capacities — the one collective of the tick, no host sync, no size
  // exchange — unless the engine was created with rg_config.wire_exact (and the transport has
  // allgather_u64): then the plan's host sync and a size all-gather, and a transfer of exactly the
  // planned bytes.
  const bool fixed = !e->c.wire_exact || !t->allgather_u64;
  const uint32_t N = e->pl.N, me = e->pl.rank;
  std::vector<uint64_t> ssize(N), soff(N), rsize(N), roff(N);
  if (fixed) {
    RGCHK(rg_wire_plan_fixed(e, ssize.data(), rsize.data()));
  } else {
    std::vector<uint64_t> all((uint64_t)N * N);
    RGCHK(rg_wire_plan(e, ssize.data()));
    if (t->allgather_u64(t->user, ssize.data(), all.data(), N) != 0)
      return fail(RG_EHIP, "rg_wire_exchange: transport allgather_u64 failed");
    for (uint32_t r = 0; r < N; ++r) {
      if (all[(uint64_t)me * N + r] != ssize[r])
        return fail(RG_EINVAL, "rg_wire_exchange: allgather returned another rank's sizes");
      rsize[r] = all[(uint64_t)r * N + me];
    }
  }
  uint64_t st = 0, rt = 0;
  for (uint32_t r = 0; r < N; ++r) {
    roff[r] = rt;
    rt += rsize[r];
  }
  // One buffer: the receive regions, then the send regions to the other ranks. The region to this
  // rank is packed where rg_wire_recv reads it (the transport moves 0 bytes for it: no self copy of
  // a rehearsal's ~2 GB); both ends of that link are this engine, so its send and
  // receive sizes agree. RAFTGPU_RCCL_SELF=rccl (tests: the transport's grouped path at one rank)
  // keeps a separate send region for it.
  const bool alias = !e->self_via_transport && ssize[me] && ssize[me] == rsize[me];
  const uint64_t sbase = (rt + 255) & ~255ull;
  for (uint32_t r = 0; r < N; ++r) {
    if (alias && r == me) {
      soff[r] = roff[r];
      continue;
    }
    soff[r] = sbase + st;
    st += ssize[r];
  }
  RGCHK(xgrow(e, &e->x_recv, &e->x_recv_cap, std::max<uint64_t>(sbase + st, 256)));
  RGCHK(wire_pack_at(e, e->x_recv, soff.data(), e->x_recv_cap, "rg_wire_exchange"));
  std::vector<uint64_t> ts(ssize), tr(rsize);
  if (alias) ts[me] = tr[me] = 0;
  if (t->alltoallv(t->user, e->x_recv, soff.data(), ts.data(), e->x_recv, roff.data(), tr.data(),
                   (void*)e->stream) != 0)
    return fail(RG_EHIP, "rg_wire_exchange: transport alltoallv failed");
  if (sent_bytes) *sent_bytes = st - (alias ? 0 : ssize[me]);
  return rg_wire_recv(e, e->x_recv, rsize.data());
}

}  // extern "C"
