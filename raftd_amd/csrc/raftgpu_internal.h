// raftgpu_internal.h — device-side layout shared by the kernels and the host runtime.
// Layout rationale: DESIGN.md §2. Replicas are numbered slot-major on the device,
// q = s·G + g (s = replica slot, g = group), so that the 64 lanes of a wave hold the same slot
// of 64 consecutive groups: every structure-of-arrays access below is coalesced, and in steady
// state the lanes of a wave take the same branch (same role).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#ifndef RG_HD_INLINE
#define RG_HD_INLINE __host__ __device__ inline
#endif

namespace rg {

constexpr uint32_t MAX_R = 8;
// term-ring / inline-term word: term | cmd_len<<36 | type<<61 | has_payload<<62 | bank<<63
// (terms < 2^36; cmd_len = the entry's Cmd bytes, 0..max_cmd_bytes (<= MAX_CMD = 16 MiB, a 25-bit
// field); has_payload ⇔ an application entry with cmd_len > 0; bank = which of the two info banks
// holds the entry's {crc, stream position}). r01–r03 kept 13 length bits (Cmds of at
// most 8,191 B); raftd hands any Cmd []byte to Update (raft/state_machine.go:126-145), so r04 moved
// the field down: 2^36 terms is 2^36 elections of one shard.
constexpr uint64_t BANK_BIT = 1ull << 63;
constexpr uint64_t PAY_BIT = 1ull << 62;
constexpr uint64_t TYPE_BIT = 1ull << 61;
constexpr uint32_t LEN_SHIFT = 36;
constexpr uint64_t TERM_MASK = (1ull << LEN_SHIFT) - 1;
constexpr uint32_t LEN_FIELD = (1u << 25) - 1;  // bits 36..60
constexpr uint32_t MAX_CMD = 1u << 24;           // the longest Cmd rg_config.max_cmd_bytes may name
RG_HD_INLINE uint32_t word_len(uint64_t w) { return (uint32_t)(w >> LEN_SHIFT) & LEN_FIELD; }
RG_HD_INLINE uint64_t len_bits(uint32_t len) { return ((uint64_t)len << LEN_SHIFT) | (len ? PAY_BIT : 0ull); }
// 16-B chunks of the payload stream an entry occupies (0: no Cmd bytes; a ConfigChange has none)
RG_HD_INLINE uint32_t word_nc(uint64_t w) { return (w & PAY_BIT) ? (word_len(w) + 15u) >> 4 : 0u; }

// ---- paged payload stream. Every replica appends its entries' Cmd bytes, each
// rounded up to 16-B chunks, to its own stream; a stream position is a u32 chunk count (modular).
// The stream is mapped through a per-replica ring of page ids pt[q][vpn & (PTS-1)] onto 4-KiB pages
// of one engine-wide pool. Pages are taken when the stream grows (pool_kernel, after the control
// step) and returned once compaction passed them (one step later, so same-launch readers of
// entries sent in the previous step are done). Positions only grow: a truncated suffix's bytes stay
// where they are (garbage until compaction passes them), so readers of an entry never race with a
// rewrite of its index.
constexpr uint32_t PAGE_LOG = 8;                        // chunks per page = 256
constexpr uint32_t PAGE_CH = 1u << PAGE_LOG;
constexpr uint32_t PAGE_BYTES = PAGE_CH * 16;           // 4 KiB
constexpr uint32_t VPN_MASK = (1u << (32 - PAGE_LOG)) - 1;  // page numbers are positions >> 8, mod 2^24
RG_HD_INLINE uint32_t vpn_of(uint32_t pos) { return pos >> PAGE_LOG; }
RG_HD_INLINE uint32_t vpn_ceil(uint32_t pos) { return (uint32_t)(((uint64_t)pos + PAGE_CH - 1) >> PAGE_LOG) & VPN_MASK; }
RG_HD_INLINE uint32_t vpn_diff(uint32_t a, uint32_t b) { return (a - b) & VPN_MASK; }
// stream capacity rule (deterministic; the oracle applies the same): an append of c chunks is
// allowed iff its last chunk's page stays within PTS pages of the lowest page still held
RG_HD_INLINE bool stream_fits(uint32_t hw, uint32_t lpg, uint32_t c, uint32_t PTS) {
  return c == 0 || vpn_diff(vpn_of(hw + c - 1u), lpg) < PTS;
}
// slab_info.x of a proposal-slab entry: SYN_OFF = the generator's Cmd (P bytes at the entry's fixed
// slab slot); otherwise the chunk offset of a caller Cmd in its slab's Cmd arena
constexpr uint32_t SYN_OFF = 0x80000000u;
// engine-wide page pool state (device memory): free-id ring [npages] consumed at head, refilled at
// tail; limit = tail as of the last bulk launch (ids below it were written by an earlier launch)
struct PoolCtl {
  unsigned long long head, tail, limit;
  uint32_t fail;       // sticky: an allocation found the pool empty (ERR_POOL, the engine is poisoned)
  uint32_t param_err;  // sticky: a control launch found a corrupt parameter block (checksum)
};
// A ConfigChange entry (TYPE_BIT, no payload) keeps its descriptor op << 4 | (slot + 1) in the
// length field; 0 = the bootstrap entries
enum : uint32_t { CC_ADD = 1, CC_REMOVE = 2 };
RG_HD_INLINE uint64_t cc_bits(uint32_t cc) { return ((uint64_t)cc << LEN_SHIFT); }

enum : uint32_t {
  M_LOCAL_TICK = 0, M_ELECTION = 1, M_LEADER_HEARTBEAT = 2, M_NOOP = 4, M_PROPOSE = 7,
  M_CHECK_QUORUM = 10, M_REPLICATE = 12, M_REPLICATE_RESP = 13, M_REQUEST_VOTE = 14,
  M_REQUEST_VOTE_RESP = 15, M_INSTALL_SNAPSHOT = 16, M_HEARTBEAT = 17, M_HEARTBEAT_RESP = 18,
  M_READ_INDEX = 19, M_READ_INDEX_RESP = 20
};
// ReadIndex state rows ([row][nrep], updated in place by the replica's own lane, touched only on
// read traffic): the leader's pending request and the read made ready in a step
// ReadIndex rows (rdst, [RD_ROWS][nrep]; dragonboat's readIndex queue): a leader's pending requests in
// arrival order (RQ_N of them: ctx, commit index at arrival, acks | requester slot << 32), and the reads
// a replica made ready in a step (RD_N of them, in order; RD_TICK = step + 1)
constexpr uint32_t RG_RQ = 4;  // = RG_READ_QUEUE (include/raftgpu.h; checked in raftgpu_engine.cpp)
enum : uint32_t {
  RQ_N,
  RQ_CTX,
  RQ_INDEX = RQ_CTX + RG_RQ,
  RQ_ACKS = RQ_INDEX + RG_RQ,
  RD_TICK = RQ_ACKS + RG_RQ,
  RD_N,
  RD_CTX,
  RD_INDEX = RD_CTX + RG_RQ,
  RD_ROWS = RD_INDEX + RG_RQ
};
enum : uint32_t { FOLLOWER = 0, CANDIDATE = 1, LEADER = 2 };
// header word 7 of a local Replicate: its n entries all carry the inline word mt[0] (raftgpu_control.h)
constexpr uint32_t RG_UNIFORM = 1;
// The header words a message of each type carries (bit w = word w: 0 type|ids|reject|nent, 1 term,
// 2 log term, 3 log index, 4 commit, 5 hint, 6 hint high, 7 src): the sender stores only these, the
// readers load only these, and a message view shows the others as 0. The steady-state types carry
// half their 64 B (r06: at C5 the outbox planes were a third of the control step's HBM bytes); the
// rare types carry all eight. Every word a handler of the type reads is in its set.
RG_HD_INLINE uint32_t hdr_words(uint32_t type, uint32_t nent = 1) {
  return type == M_REPLICATE ? (nent ? 0xBFu  // all but the hint high
                                     : 0x1Fu)  // an empty one (a commit update): no Cmd position, no src
         : type == M_REPLICATE_RESP ? 0x2Bu   // ids|reject, term, log index, hint
         : type == M_HEARTBEAT ? 0x73u        // ids, term, commit, hint, hint high (a read's context)
         : type == M_HEARTBEAT_RESP ? 0x63u   // ids, term, hint, hint high (the context echoed)
         : type == M_NOOP ? 0x03u             // ids, term
         : 0xFFu;
}
// A message count plane (cnt, rcnt: [R src][R dst][G] u32) holds the count of a pair's messages in bits
// 0..7 and, for the first four, their classes in bits 8 + 2k: which header words the receiver loads
// before it knows the type (its step reads the counts first). MC_ALL: every word and the first inline
// term (also any message a sender did not classify, e.g. rg_deliver's); the others: hdr_words of the
// class's types, no inline term. A follower's steady inbox is an empty Replicate, a Heartbeat and a
// Replicate per commit round: loading each one's own words instead of all nine cut its reads by a third.
enum : uint32_t { MC_ALL = 0, MC_HB = 1, MC_EMPTY = 2, MC_RESP = 3 };
RG_HD_INLINE uint32_t cnt_n(uint32_t c) { return c & 0xFFu; }
RG_HD_INLINE uint32_t cnt_cls(uint32_t c, uint32_t k) { return k < 4 ? (c >> (8 + 2 * k)) & 3u : (uint32_t)MC_ALL; }
RG_HD_INLINE uint32_t msg_class(uint32_t type, uint32_t nent) {
  return type == M_HEARTBEAT ? MC_HB
         : type == M_REPLICATE && !nent ? MC_EMPTY
         : type == M_REPLICATE_RESP || type == M_HEARTBEAT_RESP ? MC_RESP
         : MC_ALL;
}
// the header words a receiver loads for a class: hdr_words of its types (a response: the words a handler
// of either response reads; a heartbeat response's word 6 is only shown in message views)
RG_HD_INLINE uint32_t cls_words(uint32_t cls) {
  return cls == MC_HB ? 0x73u : cls == MC_EMPTY ? 0x1Fu : cls == MC_RESP ? 0x2Bu : 0xFFu;
}
enum : uint32_t { RETRY = 0, WAIT = 1, REPLICATE = 2, SNAPSHOT = 3 };
enum : uint32_t { ENTRY_APP = 0, ENTRY_CONFIG = 1 };
enum : uint32_t {
  ERR_CONFLICT = 1, ERR_BEYOND = 2, ERR_RING = 4, ERR_CRC = 8, ERR_EMPTY_SNAP = 16, ERR_WIRE = 32, ERR_POOL = 64,
  ERR_TERM = 128  // a campaign at term TERM_MASK (the ring word's 36-bit term field is full) was refused
};
// RG_BOUNDS (diagnostic builds): kernels printf and skip any count or offset read from memory that
// would index outside its buffer (ERR_WIRE in the replica's err word). Product builds check only
// what arrives over the wire (unpack_kernel keeps the well-formed messages of a unit).
#ifdef RG_BOUNDS
#define RG_OOB(...) printf(__VA_ARGS__)
#else
#define RG_OOB(...) ((void)0)
#endif

// state field rows ([row][nrep])
enum : uint32_t {
  S_TERM, S_VOTE, S_LEADER, S_COMMITTED, S_APPLIED, S_LAST, S_MARKER, S_MARKER_TERM, S_SNAP_INDEX,
  S_SNAP_TERM, S_CAP_BASE, S_PROCESSED,
  S_CC_HI,  // highest index a ConfigChange entry was written to (the apply scan stops there)
  S_LAST_TERM,  // the term of entry S_LAST (S_MARKER_TERM when the log is empty above the marker): the
                // step's first term lookup without a ring read (one scattered line per replica at C5)
  S64_ROWS
};
enum : uint32_t {
  S_ROLE, S_ETICK, S_HTICK, S_RAND_TO, S_RNG_CTR, S_GRANTED, S_RESPONDED, S_ACTIVE, S_ERR, S_DROPS,
  S_MEMBERS, S_SNAP_MEMBERS, S_CC_PENDING,  // membership
  S_HW,    // payload stream: next free chunk position
  S_LPG,   // lowest stream page still held (the capacity rule's base)
  S_APG,   // stream pages held up to here (exclusive): [S_LPG, S_APG)
  S_NLPG,  // control → pool_kernel: pages below this are free once the step is done (= S_LPG: none)
  S32_ROWS
};
// job rows
enum : uint32_t { J_FIRST, J_SPOS, J_SMASK, J_DMASK, J64_ROWS };
enum : uint32_t { J_META, J_SRC, J_DPOS, J32_ROWS };
// meta = n | e0 << 8 | kind << 16 | uniform << 20 | ncu << 21
RG_HD_INLINE uint32_t job_meta(uint32_t n, uint32_t e0, uint32_t kind, bool uni, uint32_t ncu) {
  return n | (e0 << 8) | (kind << 16) | (uni ? 1u << 20 : 0u) | (ncu << 21);
}
// SRC_WIRE_PROP: a proposal forwarded from another rank — its Cmds in the receive buffer like
// SRC_WIRE's entries, but with no sender CRC to verify. SRC_CMD: caller Cmds in a slab's Cmd arena.
enum : uint32_t { SRC_NONE = 0, SRC_RING = 1, SRC_SLAB = 2, SRC_WIRE = 3, SRC_WIRE_PROP = 4, SRC_CMD = 5 };
// A job is n entries [first + e0, first + n) written to this replica's log; their Cmd bytes go to its
// stream from chunk J_DPOS on, back to back; J_DMASK = per-entry destination info bank bits.
// Uniform jobs (meta bit 20): every entry is ncu chunks and the source bytes are contiguous too, so
// the bulk kernel addresses them arithmetically (the steady state); other jobs read each entry's
// source position (the bulk kernel's per-entry path).
// SRC_RING: J_SRC = the sender's replica q, J_SMASK = per-entry source info bank bits; uniform:
//   J_SPOS = the sender's stream position of message entry 0 (header word 5 of a uniform Replicate).
// SRC_SLAB (generator Cmds, P bytes each, uniform) and SRC_CMD (caller Cmds): J_SRC = slab id | row
//   slot << 16: the batch is in slab row = column (one rank) or row slot · G + column (wire engines:
//   the proposing replica's row); SRC_CMD uniform: J_SPOS = arena chunk of entry e0.
// SRC_WIRE / SRC_WIRE_PROP: the message arrived over the wire. J_SPOS = byte offset of its first
//   entry record in the receive buffer, J_SRC = its entry count n; record e = {u64 term word, u32
//   slot crc, u32 payload chunk offset} at +16e, payloads from +16n on.
// Slot CRC: the CRC-32 of the Cmd zero-padded to S·P bytes, S = ceil(len / P) (= the Cmd's CRC when
// len = S·P). The bulk kernel computes it with P-byte lane groups; crc_of_cmd converts.

// ---- placement across ranks. Replica slot s of global group g lives on rank
// (g mod N + off_c(s)) mod N, local column j = g div N, column class c = j mod (N − 1), with
// off_c(0) = 0 and off_c(s) = ((c + s − 1) mod (N − 1)) + 1: every replica of a group shares column
// j, the plane s→d of column j goes to rank k + off_c(d) − off_c(s), and over N − 1 classes a
// leader's followers sit at every other rank equally often (the busiest xGMI link carries 2/(N−1)
// of a rank's leader→follower payload instead of 1/2 with offsets s·h). Arithmetic only: no table
// that a dynamic index could push into scratch. With N < R co-location is unavoidable: followers
// s = 1.. take the N − 1 peers, then the leader's own rank, in cycles of N (p = (s − 1) mod N, p = N − 1
// → offset 0), so the leader's rank hosts ceil(R / N) replicas and fewer follower copies cross xGMI
// (R 3 at N 2: one remote follower instead of two). For N ≥ R, p < N − 1 and nothing changes.
constexpr uint32_t MAX_RANKS = 16;
struct Placement {
  uint32_t N, rank, wire_all, col_base;  // col_base: global column of local column 0
};
// j: LOCAL column (global column = col_base + j)
RG_HD_INLINE uint32_t pl_soff(const Placement& pl, uint32_t s, uint32_t j) {
  if (s == 0 || pl.N < 2) return 0;
  const uint32_t m = pl.N - 1, p = (s - 1) % pl.N;
  if (p == m) return 0;  // N < R: every N-th follower shares the leader's rank
  return ((pl.col_base + j) % m + p) % m + 1;
}
// rank offset of the plane s→d at column j (0 = co-located)
RG_HD_INLINE uint32_t pl_off(const Placement& pl, uint32_t s, uint32_t d, uint32_t j) {
  const uint32_t N = pl.N;
  return (pl_soff(pl, d, j) + N - pl_soff(pl, s, j)) % N;
}
RG_HD_INLINE bool pl_remote(const Placement& pl, uint32_t s, uint32_t d, uint32_t j) {
  return pl.wire_all || pl_off(pl, s, d, j) != 0;
}
inline Placement make_placement(uint32_t N, uint32_t rank, uint32_t wire_all, uint32_t col_base = 0) {
  Placement pl{};
  pl.N = N ? N : 1;
  pl.rank = rank;
  pl.wire_all = wire_all ? 1 : 0;
  pl.col_base = col_base;
  return pl;
}
// global group of local replica (slot s, column j) on this rank
RG_HD_INLINE uint64_t pl_group(const Placement& pl, uint32_t s, uint32_t j) {
  const uint32_t N = pl.N;
  return (uint64_t)N * (pl.col_base + j) + (pl.rank + N - pl_soff(pl, s, j) % N) % N;
}
// index of global group g in this engine's tick-input arrays (they start at its first group)
RG_HD_INLINE uint64_t pl_input_index(const Placement& pl, uint64_t g) { return g - (uint64_t)pl.N * pl.col_base; }
// rank hosting slot s of global group g (g within this engine's columns)
RG_HD_INLINE uint32_t pl_rank_of(const Placement& pl, uint64_t g, uint32_t s) {
  const uint32_t N = pl.N;
  return (uint32_t)((g % N + pl_soff(pl, s, (uint32_t)(g / N - pl.col_base))) % N);
}

// TickParams reaches control_kernel through a pointer (a device slot, not kernel arguments), so its
// pointer fields are loaded from memory: declared in the global address space on the device, they
// keep every access a global_load / global_store instead of a flat one (same bits and layout as
// the host's plain pointers)
#if defined(__HIP_DEVICE_COMPILE__)
#define RG_G(T) __attribute__((address_space(1))) T*
#else
#define RG_G(T) T*
#endif
struct TickParams {
  uint32_t G, R, nrep, L, P, E, K, nslab, J;
  uint32_t ET, HT, CQ, SE, CO, drop_ppm, flags;
  uint32_t wire;           // wire engine: slab rows per replica (q), else per column (g)
  uint32_t AF;             // apply feedback: applied moves only by rg_notify_applied
  uint32_t PTS;            // stream pages per replica (power of two; the capacity rule)
  uint32_t JS;             // join slots (rg_config.join_slots): bootstrap with an empty log, no membership
  uint64_t seed, tick;
  Placement pl;
  // replica state, one copy updated in place: a step reads its replica's rows and writes back only
  // the fields it changed (the fast step: DESIGN.md §3 "In-place state"; r05 and earlier ping-ponged
  // two copies and copied every unchanged field through)
  RG_G(uint64_t) s64;           // [S64_ROWS][nrep]
  RG_G(uint32_t) s32;           // [S32_ROWS][nrep]
  RG_G(uint64_t) rem;           // [3][R][nrep]: match, next, rsnap
  RG_G(uint8_t) rst;            // [R][nrep]
  RG_G(uint64_t) tr;            // term ring [L][nrep]
  RG_G(const uint64_t) hdr_in;  // [8][R src][R dst][K][G]
  RG_G(uint64_t) hdr_out;
  RG_G(const uint64_t) mt_in;   // [R src][R dst][K][E][G]
  RG_G(uint64_t) mt_out;
  RG_G(const uint32_t) cnt_in;  // [R src][R dst][G]
  RG_G(uint32_t) cnt_out;
  // remote inbox (planes whose sender lives on another rank, written by unpack_kernel; same
  // layout as hdr/mt/cnt; hdr word 7 of a Replicate = byte offset of its records in the wire)
  RG_G(const uint64_t) rhdr;
  RG_G(const uint64_t) rmt;
  RG_G(const uint32_t) rcnt;
  RG_G(uint64_t) feed;          // [nrep] the step's hand-off word (feed_*, below; NULL: skip)
  RG_G(uint32_t) prof;          // RG_CTL_PROFILE builds only: [6][nrep] s_memtime stamps per phase
  RG_G(uint64_t) job64;         // [J64_ROWS][J][nrep]
  RG_G(uint32_t) job32;         // [J32_ROWS][J][nrep]
  RG_G(uint32_t) jcnt;          // [nrep]
  RG_G(const uint8_t) prop_target;
  RG_G(const uint32_t) prop_count;
  RG_G(const uint64_t) prop_hmask;  // caller proposals: entries with a non-empty Cmd (NULL: synthetic, all of len P)
  RG_G(const uint2) prop_cmd;       // caller proposals: {stream chunks | contiguous << 31, arena chunk of entry 0}
  RG_G(const uint2) slab_info;      // [nslab][rows][E] {0, Cmd length} of the proposal slabs
  RG_G(const uint8_t) campaign;
  RG_G(const uint8_t) isolate;
  RG_G(const uint64_t) read_ctx;    // [global rid] ReadIndex request contexts of this tick (NULL: none)
  RG_G(const uint16_t) cc_in;       // [global group] membership change of this tick: slot | descriptor << 8 (0 none)
  uint32_t IM;                 // bootstrap membership (rg_config.initial_members, 0 read as every slot)
  RG_G(uint64_t) rdst;              // [RD_ROWS][nrep] ReadIndex state
  RG_G(const uint2) info;           // [2 banks][nrep][L] {slot crc, stream position} (a freed stream's bound)
  RG_G(PoolCtl) pool;               // sticky param_err on a checksum mismatch
  // the fast path's hand-off: control_fast_kernel appends a replica whose step left the
  // fast path to slow_flag (a list: slow_cnt[tick & 1] of them, one atomic per wave), and
  // control_slow_kernel re-runs those steps, a grid-stride walk of the list (r06: it was a flag per
  // replica and a full grid, 0.05 ms at C5 for a handful of lanes). slow_cnt[(tick + 1) & 1] is zeroed
  // by the fast launch (its readers are done). Diagnostic 2-D builds (RG_AB_CTL2D) keep the flags.
  RG_G(uint32_t) slow_cnt;          // [2] (NULL: no fast path; control_kernel steps every replica)
  RG_G(uint32_t) slow_flag;         // [nrep]: the hand-off list (RG_AB_CTL2D: a flag per replica)
  uint64_t csum;                    // tp_checksum of every word above (host-computed, checked first)
};
// the parameter block's checksum: Σ_i tp_mix(word_i + (i + 1)·φ) mod 2^64 over its words before `csum`
// (a stale or torn block is reported as an engine error instead of being dereferenced).
// A sum, not a chain, so a wave checks it with one coalesced load (lane i, word i) and a reduction.
RG_HD_INLINE uint64_t tp_mix(uint64_t z) {
  z ^= z >> 31;
  z *= 0x9E3779B97F4A7C15ULL;
  return z ^ (z >> 29);
}
RG_HD_INLINE uint64_t tp_term(uint64_t word, uint32_t i) { return tp_mix(word + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL); }
constexpr uint32_t TP_WORDS = (uint32_t)(offsetof(TickParams, csum) / 8);
static_assert(TP_WORDS <= 64, "the checksum is verified with one word per lane of a wave");

struct BulkParams {
  uint32_t G, R, nrep, L, P, E, J, crc_const, tile;  // tile: groups per wave work item (1..64)
  uint32_t wire_mode;    // wire engine (ranks > 1 or wire_all): SRC_WIRE jobs, one slab row per replica
  const uint64_t* job64;
  const uint32_t* job32;
  const uint32_t* jcnt;
  const uint64_t* tr;    // term ring [L][nrep] (per-entry Cmd lengths of non-uniform jobs)
  uint2* info;           // [2 banks][nrep][L] {slot crc, stream position}
  uint8_t* pool;         // [npages][4 KiB] payload pages
  uint32_t PTS;          // page-table entries per replica; pt = the kernel's own argument
  const uint8_t* slabs;  // [nslab][rows][E][P], rows = G, or nrep in wire_mode (generator Cmds)
  const uint2* slab_info;  // [nslab][rows][E] {SYN_OFF or arena chunk, len}
  const uint8_t* cmds;   // [nslab][cmd_cap] caller Cmd arenas
  uint64_t cmd_cap;
  const uint8_t* wire;   // receive buffer of the last exchange (SRC_WIRE jobs)
  uint32_t* crc_err;     // [nrep] sticky ERR_CRC from payload verification
  const uint32_t* crc_tab;
  PoolCtl* poolctl;      // block 0 publishes limit = tail (the pool kernel of this tick has run)
  uint64_t wire_bytes;   // bytes of `wire` in use (job bounds checks)
  uint32_t nslab;
  uint32_t multijob;     // small jobs share a ring pass (bulk_kernel<.., MJ>; the engine's choice)
  uint32_t small;        // bulk_small_kernel ran first: bulk_kernel skips the replicas it took (small_job)
  uint32_t* rest;        // [ceil(G / 64) * R] per 64-group block and slot: 1 if bulk_small_kernel left a
                         // replica with jobs there (bulk_kernel skips the tiles of a block it took whole)
  uint64_t* rest_tick;   // bulk_small_kernel stamps `tick` here if it left any replica to bulk_kernel; a
  uint64_t tick;         //   bulk_kernel that finds another stamp has nothing to do and exits at once
                         //   (C5: every block taken whole; the launch was 0.096 ms of LDS staging and tile walks)
  uint32_t wg_waves;     // waves per bulk_kernel workgroup (1..4)
};

// pool_kernel (after control, before bulk): frees the stream pages control released, allocates the
// pages the step's appends need, and updates S_LPG / S_APG; on an empty pool ERR_POOL + no jobs
struct PoolParams {
  uint32_t nrep, PTS;
  uint64_t npages;
  uint32_t* s32;               // state rows: S_HW, S_NLPG (control's) in; S_LPG / S_APG out
  uint32_t* pt;                // [nrep][PTS] page ids
  uint32_t* fring;             // [npages] free page ids
  PoolCtl* ctl;
  uint32_t* jcnt;              // the step's job counts (zeroed for a replica whose allocation failed)
};

// CRC-32/IEEE tables: T[k][b] = raw CRC of byte b followed by k zero bytes (k = 0..15);
// S[j][q][b] = the raw state (b << 8q) advanced through 16·2^j zero bytes (j = 0..5).
// CRC-32 tables (device copy in BulkParams::crc_tab, staged into LDS by bulk_kernel):
//   T  [16][256]  slice-by-16: T[m][b] = raw CRC of byte b followed by m zero bytes
//   N  [16][2][16] the same split into nibbles (lo, hi) — conflict-free 16-word LDS tables
//   SH [NCH][8][16] (row stride CRC_SH_STRIDE) per-lane shift: SH[c][j][n] = raw CRC of nibble n
//      at bit 4j of a 32-bit CRC state followed by 16·(NCH−1−c) zero bytes, NCH = P/16
//   ZI [10][8][16] (global memory only, after SH) inverse shifts: ZI[b][j][n] = nibble n at bit 4j of
//      a raw state moved back through 2^b zero bytes (Z^-(2^b)); crc_of_cmd uses them
constexpr uint32_t CRC_T_WORDS = 16 * 256;
constexpr uint32_t CRC_N_WORDS = 16 * 2 * 16;
constexpr uint32_t CRC_SH_STRIDE = 8 * 16 + 2;  // +2 words: lanes' tables start on different banks
constexpr uint32_t CRC_SH_MAX_WORDS = 64 * CRC_SH_STRIDE;
constexpr uint32_t CRC_ZI_BITS = 10;  // S·P − len < P <= 1024
constexpr uint32_t CRC_ZI_WORDS = CRC_ZI_BITS * 8 * 16;
constexpr uint32_t CRC_ZI_OFF = CRC_T_WORDS + CRC_N_WORDS + CRC_SH_MAX_WORDS;
// ZP [8][16]: Z^P (P zero bytes) on a raw state, to chain the P-byte segments of a Cmd longer than P
// (the chain starts from the init value ~0, so no per-length finalisation constant is needed)
constexpr uint32_t CRC_ZP_OFF = CRC_ZI_OFF + CRC_ZI_WORDS;
constexpr uint32_t CRC_ZP_WORDS = 8 * 16;
// 16 zero bytes (16-B aligned): where the bulk kernel's idle lanes load from, so a lane past its
// entry's chunks adds nothing to the lane group's CRC
constexpr uint32_t CRC_ZERO_OFF = (CRC_ZP_OFF + CRC_ZP_WORDS + 3) & ~3u;
constexpr uint32_t CRC_TAB_WORDS = CRC_ZERO_OFF + 4;

// CRC-32 of a Cmd of len bytes from its slot CRC (the CRC of the Cmd zero-padded to S·P bytes,
// S = ceil(len / P)): slot = cs ^ raw(slot), raw(slot) = Z^(S·P−len) raw(Cmd), so
// crc(Cmd) = Z^-(S·P−len)(slot ^ ~0) ^ ~0 (init / xorout ~0; Z = one zero byte, invertible).
RG_HD_INLINE uint32_t crc_of_cmd(uint32_t slot_crc, uint32_t len, uint32_t P, const uint32_t* zi) {
  if (!len) return 0;
  const uint32_t padded = (len + P - 1) / P * P;
  if (len == padded) return slot_crc;
  uint32_t v = slot_crc ^ 0xFFFFFFFFu;
  const uint32_t k = padded - len;
  for (uint32_t b = 0; b < CRC_ZI_BITS; ++b) {
    if ((k >> b) & 1u) {
      uint32_t r = 0;
      for (uint32_t j = 0; j < 8; ++j) r ^= zi[(b * 8 + j) * 16 + ((v >> (4 * j)) & 0xF)];
      v = r;
    }
  }
  return v ^ 0xFFFFFFFFu;
}

// byte offset in the pool of chunk `pos` of replica q's payload stream
RG_HD_INLINE uint64_t stream_byte(const uint32_t* pt, uint32_t PTS, uint32_t q, uint32_t pos) {
  const uint32_t pid = pt[(uint64_t)q * PTS + (vpn_of(pos) & (PTS - 1u))];
  return ((uint64_t)pid * PAGE_BYTES) + ((uint64_t)(pos & (PAGE_CH - 1u)) << 4);
}

// host-side launchers (raftgpu_kernels.hip)
// control_kernel<R> over nrep lanes; *p: the tick's parameter block in device memory
hipError_t launch_control(const TickParams* p, uint32_t* perr, uint32_t R, uint32_t nrep, hipStream_t s);
// the fast path: control_fast_kernel<R> over every replica, then control_slow_kernel<R> over the replicas
// it handed off (the parameter block's slow_cnt / slow_flag)
hipError_t launch_control_fast(const TickParams* p, uint32_t* perr, uint32_t R, uint32_t nrep, bool fb, hipStream_t s);
// k ticks of a metadata-only one-rank engine in one launch (p = k consecutive sealed blocks)
hipError_t launch_control_resident(const TickParams* p, uint32_t k, uint32_t* perr, uint32_t R, uint32_t G,
                                   hipStream_t s);
// one instantiation per translation unit (raftgpu_ctl.hip -DRG_CTL_R, raftgpu_bulk.hip -DRG_BULK_W/MJ)
template <int R>
hipError_t launch_control_t(const TickParams* p, uint32_t* perr, uint32_t nrep, hipStream_t s);
template <int R>
hipError_t launch_control_fast_t(const TickParams* p, uint32_t* perr, uint32_t nrep, bool fb, hipStream_t s);
template <int R>
hipError_t launch_control_resident_t(const TickParams* p, uint32_t k, uint32_t* perr, uint32_t G, hipStream_t s);
template <bool W, bool MJ>
hipError_t launch_bulk_t(const BulkParams& p, const uint32_t* pt, hipStream_t s, int grid);
template <bool W, bool MJ>
int bulk_occupancy_t(uint32_t P);
hipError_t launch_pool(const PoolParams& p, hipStream_t s);
// every page free, every replica's stream empty (bootstrap)
hipError_t launch_pool_reset(uint32_t* fring, uint64_t npages, PoolCtl* ctl, hipStream_t s);
hipError_t launch_bulk(const BulkParams& p, const uint32_t* pt, hipStream_t s, int grid);
hipError_t launch_bootstrap(const TickParams& p, uint2* info, hipStream_t s);
// the address of a launch's kernel-argument segment (where the runtime put the arguments)
hipError_t launch_kernarg_probe(uint64_t* out, uint64_t tag, hipStream_t s);
// synthetic Cmds into slabs [slab0, slab0 + nslab)
hipError_t launch_fill_slabs(uint8_t* slabs, uint2* slab_info, uint32_t slab0, uint32_t nslab, uint32_t G, uint32_t rows,
                             uint32_t E, uint32_t P, uint64_t seed, const Placement& pl, hipStream_t s);
// caller proposals (rg_propose): the Cmd bytes reach their slab's arena by one H2D copy; this
// writes their descriptors slab_info[info_at[e]] = {chunk[e], len[e]}
struct StageParams {  // rg_propose: one row per batch; the kernel expands the batch's Cmds from lens
  uint2* slab_info;
  const uint64_t* info_at;  // [n] slab_info index of the batch's first Cmd
  const uint64_t* first;    // [n] index of its first Cmd in lens
  const uint32_t* chunk;    // [n] arena chunk of its first Cmd (within the slab's arena)
  const uint32_t* count;    // [n] Cmds (1..64)
  const uint32_t* lens;     // the call's lens[]
  uint8_t* arena;           // the slab's Cmd arena (padding of short Cmds zeroed here)
  uint64_t n;
};
hipError_t launch_stage_cmds(const StageParams& a, hipStream_t s);
hipError_t launch_probe_copy(const void* src, void* dst, uint64_t bytes, hipStream_t s);
// device staging → host-mapped pinned memory with a few workgroups (rg_apply_async)
hipError_t launch_copy_to_host(const void* src, void* dst, uint64_t bytes, hipStream_t s);
hipError_t launch_sum_committed(const TickParams& p, unsigned long long* out, hipStream_t s);
hipError_t launch_traffic(const TickParams& p, unsigned long long* out6, hipStream_t s);
// committed-entry copy-back (raftgpu_apply.hip): after a tick, the application entries each replica
// handed over in it, [apply_lo, processed] (feed_apply_lo), gathered for IOnDiskStateMachine.Update as runs of
// consecutive indices (rg_apply_run) + a {len, crc} per entry (rg_apply_cmd); payloads packed back
// to back, each rounded up to 16 B
struct ApplyParams {
  uint32_t G, R, nrep, L, P;
  uint32_t slot_mask;       // replicas whose slot bit is set
  Placement pl;
  const uint64_t* s64;      // current state (applied)
  const uint64_t* feed;     // the last step's hand-off words (its apply window)
  const uint64_t* tr;
  const uint2* info;
  const uint8_t* pool;
  const uint32_t* pt;
  uint32_t PTS;
  const uint32_t* zi;       // CRC inverse-shift tables (crc_of_cmd)
  uint32_t* cnt;            // [nrep] entries per replica
  uint32_t* ccnt;           // [nrep] payload chunks per replica
  uint32_t* rcnt;           // [nrep] runs per replica
  uint64_t* off;            // [nrep + 1] exclusive scan of cnt
  uint64_t* coff;           // [nrep + 1] exclusive scan of ccnt
  uint64_t* roff;           // [nrep + 1] exclusive scan of rcnt
  uint64_t* bsum;           // scan scratch
  uint8_t* out_run;         // [runs] rg_apply_run (device staging)
  uint8_t* out_cmd;         // [n] rg_apply_cmd
  uint8_t* out_pay;         // [chunks][16]; NULL: by reference (no Cmd bytes; rg_get_update with
                            // RG_UPDATE_PERSIST: the host holds every committed Cmd from a persist section)
};
hipError_t launch_apply_count(const ApplyParams& a, uint64_t* totals /*[3]: entries, chunks, runs*/, hipStream_t s);
// The step's hand-off word per replica (one 8-byte store; rg_get_update reads it with the state rows):
//   bits 0..31   apply window length n: entries (processed - n, processed] went to the state machine
//   bits 32..60  persist back b: entries [last - b + 1, last] were written in the step (0: none)
//   bit 61       a snapshot was restored at processed - n (the apply window starts above it)
//   bit 62       persist: the step wrote entries or changed the hard state (term, vote, commit, last,
//                marker or snapshot index) — with state in place there is no previous copy to diff
//   bit 63       the step took a snapshot
// All zero (bootstrap, an imported replica until it steps): nothing to apply, persist or report.
// The lengths fit: a step applies and writes at most log_capacity (<= 2^28) entries.
constexpr uint64_t FEED_RESTORED = 1ull << 61, FEED_PERSIST = 1ull << 62, FEED_TAKEN = 1ull << 63;
RG_HD_INLINE uint64_t feed_word(uint64_t processed, uint64_t apply_from, uint64_t last, uint64_t wlo,
                                bool persist, bool restored, bool took) {
  return (processed - apply_from) | (wlo <= last ? (last - wlo + 1) << 32 : 0ull) |
         (restored ? FEED_RESTORED : 0ull) | (persist ? FEED_PERSIST : 0ull) | (took ? FEED_TAKEN : 0ull);
}
RG_HD_INLINE uint64_t feed_apply_lo(uint64_t f, uint64_t processed) { return processed - (uint32_t)f + 1; }
RG_HD_INLINE uint64_t feed_restored_at(uint64_t f, uint64_t processed) {
  return (f & FEED_RESTORED) ? processed - (uint32_t)f : 0ull;
}
// the lowest index written (~0: none, the entry window [lo, last] is empty)
RG_HD_INLINE uint64_t feed_persist_lo(uint64_t f, uint64_t last) {
  const uint64_t b = (f >> 32) & ((1ull << 29) - 1);
  return b ? last - b + 1 : ~0ull;
}
// snapshot events (raftgpu_apply.hip)
struct SnapParams {
  uint32_t G, R, nrep, slot_mask;
  Placement pl;
  const uint64_t* s64;      // current state (snap_index, snap_term, processed)
  const uint64_t* feed;     // the last step's hand-off words (FEED_RESTORED / FEED_TAKEN)
  const uint64_t* rdst;     // ReadIndex state (read results)
  uint64_t tick;            // the ticks run so far (a read made ready in the last one has RD_TICK == tick)
  uint32_t* cnt;
  uint64_t* off;
  uint64_t* bsum;
  uint8_t* out;             // [n] rg_snapshot_event
};
hipError_t launch_snap_count(const SnapParams& a, uint64_t* total, hipStream_t s);
hipError_t launch_snap_gather(const SnapParams& a, hipStream_t s);
// reads made ready in the last tick (rg_read_index_results), same count / scan / gather shape
hipError_t launch_read_count(const SnapParams& a, uint64_t* total, hipStream_t s);
hipError_t launch_read_gather(const SnapParams& a, hipStream_t s);
// persistence copy-back (raftgpu_apply.hip): per replica whose log or hard state changed in the
// last tick, its state record and the entries it rewrote ([persist_lo, last]); full = every
// replica with its whole log window (marker, last] (a checkpoint). Payloads packed (rg_persist_entry.off)
struct PersistParams {
  uint32_t G, R, nrep, L, P, full;
  uint32_t slot_mask;        // replicas whose slot bit is set (a node's replicas; rg_persist_collect: all)
  Placement pl;
  const uint64_t* s64;       // current state
  const uint32_t* s32;       // current state (membership)
  const uint64_t* feed;      // the last step's hand-off words (FEED_PERSIST, the entries written)
  const uint64_t* tr;
  const uint2* info;
  const uint8_t* pool;
  const uint32_t* pt;
  uint32_t PTS;
  const uint32_t* zi;
  uint32_t* scnt;            // [nrep] 1 if the replica has a record
  uint32_t* ecnt;            // [nrep] entries to save
  uint32_t* ccnt;            // [nrep] their payload chunks
  uint32_t* tcnt;            // [nrep] their term runs
  uint64_t* soff;            // [nrep + 1]
  uint64_t* eoff;            // [nrep + 1]
  uint64_t* coff;            // [nrep + 1]
  uint64_t* toff;            // [nrep + 1]
  uint64_t* bsum;
  uint8_t* out_state;        // [ns] rg_persist_state
  uint8_t* out_ent;          // [ne] rg_persist_entry (8 B: len, crc)
  uint8_t* out_term;         // [nt] rg_persist_term
  uint8_t* out_pay;          // [chunks][16]
};
hipError_t launch_persist_count(const PersistParams& a, uint64_t* totals /*[4]: states, entries, chunks, terms*/,
                                hipStream_t s);
hipError_t launch_persist_gather(const PersistParams& a, hipStream_t s);
hipError_t launch_apply_gather(const ApplyParams& a, uint64_t nruns, hipStream_t s);
// exclusive scan of n u32 into out[0..n] (out[n] = total); bsum: (n + 1023) / 1024 + 1 words
hipError_t launch_scan_u32(const uint32_t* in, uint32_t n, uint64_t* bsum, uint64_t* out, hipStream_t s);

// admin gathers / scatters behind the read / import / deliver entry points (raftgpu_admin.hip)
struct AdminParams {
  TickParams t;              // the parameter block the next tick would use (s64_in = current state)
  const uint2* info;
  uint8_t* pool;
  uint32_t* pt;
  uint32_t PTS;
  uint32_t row;              // bytes per entry row of rg_read_entries / rg_import_replica (max_cmd_bytes)
  uint32_t* fring;
  uint64_t npages;
  PoolCtl* poolctl;
  const uint32_t* crc_err;
  const uint32_t* zi;
};
hipError_t launch_gather_replicas(const AdminParams& a, uint32_t first_rid, uint32_t n, void* out_views,
                                  hipStream_t s);
hipError_t launch_gather_msgs(const AdminParams& a, uint32_t rid, uint32_t dst, void* out_hdr, uint64_t* out_terms,
                              uint32_t* out_cnt, hipStream_t s);
hipError_t launch_gather_entries(const AdminParams& a, uint32_t rid, uint64_t first, uint32_t n, void* out_views,
                                 hipStream_t s);
// the Cmds of entries first .. first+n-1 of rid: entry i's whole chunks to out + ao[i] (ao[i] = ~0: none)
hipError_t launch_gather_cmds(const AdminParams& a, uint32_t rid, uint64_t first, uint32_t n, const uint64_t* ao,
                              uint8_t* out, hipStream_t s);
// import: the view + entry words (term|len|type|pay, bank 0) + slot CRCs + stream positions of a fresh
// stream (chunk offsets from 0) + the Cmds back to back in whole chunks (nch in all). The replica's
// old stream pages go back to the pool and its new stream takes ceil(nch / 256) pages (*status = 1
// if the pool is empty: nothing changed)
hipError_t launch_scatter_replica(const AdminParams& a, uint32_t rid, const void* view, const uint64_t* words,
                                  const uint32_t* crcs, const uint32_t* pos, const uint8_t* chunks, uint32_t nent,
                                  uint32_t nch, uint32_t* status, hipStream_t s);
hipError_t launch_deliver(const AdminParams& a, uint32_t rid_src, const void* hdr, uint32_t* status,
                          hipStream_t s);
// rg_notify_applied: check (pass 0: *bad = number of rids / indices out of range) or set (pass 1) applied
// rg_compact: every replica of global shard `group` hosted here compacts to min(index, its snap_index)
// when that is above its marker; *n (device, zeroed by the caller) counts them
hipError_t launch_compact(const AdminParams& a, uint64_t group, uint64_t index, uint32_t* n, hipStream_t s);
hipError_t launch_notify_applied(const AdminParams& a, const uint32_t* rids, const uint64_t* index, uint32_t n,
                                 int pass, uint32_t* bad, hipStream_t s);
// rg_digest: out[0] += Σ view chains, out[1] += Σ log chains (out zeroed by the caller)
hipError_t launch_digest(const AdminParams& a, unsigned long long* out, hipStream_t s);
// rg_commit_update(RG_COMMIT_APPLIED): applied = processed for every replica of the slot mask
hipError_t launch_applied_all(const AdminParams& a, uint32_t slot_mask, hipStream_t s);
int bulk_lds_bytes(uint32_t P);
int bulk_blocks_per_cu(uint32_t P);

}  // namespace rg
