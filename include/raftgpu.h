/*
 * raftgpu.h — C-ABI of the MI355X batched Raft step engine (raftd-amd).
 *
 * The engine is the batched analogue of dragonboat v4's internal/raft `Peer`
 * (Launch/Handle/Tick/GetUpdate/Commit), for every replica of every group that one process
 * hosts, resident in MI355X HBM. raftd reaches that code only through dragonboat's NodeHost,
 * which offers no plugin point for the raft step, so these entry points are what
 * a raftd-side cgo shim re-implementing the NodeHost subset binds:
 *
 *   rg_create / rg_destroy        ← dragonboat.NewNodeHost / NodeHost.Close
 *                                    (/root/reference/raft/raft_manager.go:102-109, :159)
 *   rg_bootstrap                  ← NodeHost.StartOnDiskReplica(initialMembers, join=false, …, rc)
 *                                    (raft_manager.go:142-144; rc = ElectionRTT 10, HeartbeatRTT 1,
 *                                    CheckQuorum, SnapshotEntries 1000, CompactionOverhead 5 at :92-100)
 *   rg_tick / rg_tick_device      ← the NodeHost tick goroutine (RTTMillisecond 3, raft_manager.go:105)
 *                                    driving Peer.Tick + Peer.Handle for all shards
 *   rg_propose                    ← NodeHost.Propose / SyncPropose(session, cmd []byte) → Peer.ProposeEntries:
 *                                    the client command bytes raftd's state machine later receives
 *                                    verbatim as statemachine.Entry.Cmd (raft/state_machine.go:126-145)
 *   rg_leader                     ← NodeHost.GetLeaderID (raft/members.go:21)
 *   rg_read_replicas              ← NodeHost.SyncGetShardMembership / raftState (raft/members.go:30)
 *   rg_read_entries               ← committed-range copy-back feeding IOnDiskStateMachine.Update
 *                                    (raft/state_machine.go:136-166)
 *   rg_deliver                    ← transport delivery of a pb.Message from another host
 *
 * Conventions: plain pointers and sizes; every call returns RG_OK (0) or a negative RG_E*
 * code, with rg_last_error() (thread-local) describing the failure. An engine handle is not
 * thread-safe: one host thread drives it, as one dragonboat step worker owns a shard.
 * The engine owns all device memory. Step semantics: DESIGN.md §1.
 */
#ifndef RAFTGPU_H
#define RAFTGPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RG_MAX_REPLICAS 8

enum {
  RG_OK = 0,
  RG_EINVAL = -1,      /* bad argument or configuration */
  RG_ENOMEM = -2,      /* device allocation failed */
  RG_EFULL = -3,       /* a bounded buffer is full (e.g. rg_deliver into a full slot) */
  RG_EHIP = -4,        /* HIP runtime error */
  RG_EINVARIANT = -5   /* a dragonboat plog.Panicf invariant fired (see rg_replica_view.err) */
};

/* message types (raftpb.MessageType numbering as recalled) */
enum {
  RG_MSG_NOOP = 4, RG_MSG_PROPOSE = 7, RG_MSG_REPLICATE = 12, RG_MSG_REPLICATE_RESP = 13,
  RG_MSG_REQUEST_VOTE = 14, RG_MSG_REQUEST_VOTE_RESP = 15, RG_MSG_INSTALL_SNAPSHOT = 16,
  RG_MSG_HEARTBEAT = 17, RG_MSG_HEARTBEAT_RESP = 18, RG_MSG_READ_INDEX = 19, RG_MSG_READ_INDEX_RESP = 20
};
enum { RG_FOLLOWER = 0, RG_CANDIDATE = 1, RG_LEADER = 2 };
enum { RG_REMOTE_RETRY = 0, RG_REMOTE_WAIT = 1, RG_REMOTE_REPLICATE = 2, RG_REMOTE_SNAPSHOT = 3 };
enum { RG_ENTRY_APPLICATION = 0, RG_ENTRY_CONFIG_CHANGE = 1 };
/* rg_import_replica types[] flag: an application entry with an empty Cmd (a leader's no-op),
 * stored without payload even when payloads are given (WAL restore) */
#define RG_ENTRY_EMPTY 0x100u
enum {
  RG_ERR_CONFLICT_COMMITTED = 1, RG_ERR_COMMIT_BEYOND_LAST = 2, RG_ERR_RING_FULL = 4,
  RG_ERR_CRC = 8, RG_ERR_EMPTY_SNAPSHOT = 16,
  RG_ERR_MALFORMED = 32, /* a message with an impossible sender / destination was ignored */
  RG_ERR_POOL = 64,      /* the payload page pool was empty: this replica's appends of a step were lost */
  RG_ERR_TERM_LIMIT = 128 /* a campaign at term 2^36 - 1 was refused: terms are 36-bit (the ring word
                             holds the Cmd length beside the term); the replica stays a
                             follower at that term. ~6.9e10 elections: unreachable in service */
};
#define RG_TICK_NO_LOCALTICK 1u

typedef struct rg_config {
  uint32_t groups;              /* shards hosted by this engine */
  uint32_t replicas;            /* replicas per shard, IDs 1..replicas (1..8) */
  uint32_t log_capacity;        /* log ring entries per replica (power of two) */
  uint32_t payload_bytes;       /* Cmd lane-group size P (bytes): 0 (metadata only) or a power of two in
                                   [16, 1024]; the size of the generator's synthetic Cmds. Caller Cmds
                                   are 0..max_cmd_bytes bytes (below) */
  uint32_t max_entries_per_msg; /* entries per Replicate / proposal batch (1..64) */
  uint32_t max_msgs_per_pair;   /* messages per (replica, destination) per tick (1..16) */
  uint32_t num_slabs;           /* proposal payload slabs, tick t uses slab t % num_slabs (>= 2) */
  uint32_t election_rtt;        /* config.Config.ElectionRTT (raftd: 10) */
  uint32_t heartbeat_rtt;       /* config.Config.HeartbeatRTT (raftd: 1) */
  uint32_t check_quorum;        /* config.Config.CheckQuorum (raftd: true) */
  uint32_t snapshot_entries;    /* config.Config.SnapshotEntries (raftd: 1000; 0 = off) */
  uint32_t compaction_overhead; /* config.Config.CompactionOverhead (raftd: 5) */
  uint32_t drop_ppm;            /* deterministic message loss, parts per million (tests) */
  int32_t device;               /* HIP device ordinal */
  uint64_t seed;
  /* Placement across ranks (one engine per GPU). Replica slot s of global group g
   * lives on rank (g mod ranks + off(s, g div ranks)) mod ranks, off(0) = 0, off(s) = ((j mod
   * (ranks-1)) + s - 1) mod (ranks-1) + 1, so with ranks >= replicas every replica of a group is
   * on a different GPU and followers spread evenly over the other ranks. An engine hosts
   * `groups` local columns; the shard set is ranks·groups global groups. Tick inputs are indexed
   * by GLOBAL group / replica id. ranks = 0 is read as 1. */
  uint32_t ranks;               /* 1..16 */
  uint32_t rank;                /* this engine's rank */
  uint32_t wire_all;            /* tests: send co-located messages through the wire too */
  uint32_t column_base;         /* global column of local column 0: a rank may host several engines
                                   over disjoint column ranges (their tick-input arrays then start
                                   at global group ranks·column_base) */
  uint32_t crc32c;              /* entry checksum: 0 = CRC-32/IEEE (zlib's, default), 1 = CRC-32C
                                   (Castagnoli, as pebble/tan WAL records use) */
  uint32_t apply_feedback;      /* 0: `applied` follows `processed` at the end of every tick (the state
                                   machine keeps up); 1: it moves only by rg_notify_applied
                                   (dragonboat's NotifyRaftLastApplied, raft/state_machine.go:101-166) */
  uint32_t initial_members;     /* bootstrap voting membership, bit s = slot s: StartOnDiskReplica's
                                   initialMembers (raft/raft_manager.go:114-144); 0 = every slot */
  /* Cmd storage: every replica appends its entries' Cmds, each at its own length
   * rounded up to 16 B, to a payload stream mapped onto 4-KiB pages of one engine-wide pool. */
  uint32_t max_cmd_bytes;       /* longest Cmd (raft/state_machine.go:126-145 hands any Cmd []byte back):
                                   payload_bytes .. 16 MiB (16,777,216); 0 = payload_bytes. payload_bytes
                                   is the Cmd size the payload kernel's lane groups and the benchmark's
                                   synthetic Cmds use; longer Cmds take several groups. Terms are < 2^36
                                   (the Cmd length shares the term word) */
  uint32_t stream_pages;        /* pages one replica's live stream may span (power of two); an append
                                   beyond it is refused like one beyond log_capacity.
                                   0 = twice a full log of payload_bytes Cmds, plus room for two of the
                                   longest Cmds (2·(ceil(max_cmd_bytes / 4096) + 1) pages) when
                                   max_cmd_bytes > payload_bytes, rounded up to a power of two */
  uint32_t pool_pages;          /* 4-KiB pages in the pool (<= 2^24); 0 = a full log of payload_bytes
                                   Cmds per replica, capped at 2^24. An empty pool poisons the engine:
                                   RG_ERR_POOL in the affected replicas, rg_pool_stats().fail */
  uint32_t join_slots;          /* slots started by StartOnDiskReplica(join = true) (raft_manager.go:
                                   134-144): empty log, term 0, not a member until a ConfigChange that
                                   adds them reaches them; 0 = none */
  uint32_t wire_exact;          /* rg_wire_exchange region sizing: 0 = fixed capacities (one collective per
                                   tick, no host sync; the default), 1 = exact sizes (a plan host sync and
                                   a size all-gather through the transport first) */
} rg_config;

typedef struct rg_replica_view {
  uint64_t term, vote, leader, committed, applied, last, marker, marker_term;
  uint64_t snap_index, snap_term, cap_base;
  uint64_t processed; /* committed entries handed to the state machine (entryLog.processed) */
  uint32_t role, election_tick, heartbeat_tick, rand_timeout, rng_ctr;
  uint32_t granted, responded, active, err, drops;
  uint32_t members;      /* voting membership as this replica applied it, bit s = slot s */
  uint32_t snap_members; /* the membership its latest snapshot records */
  uint32_t cc_pending;   /* leader: a config change is in flight (pendingConfigChange) */
  uint32_t _mpad;
  uint64_t match[RG_MAX_REPLICAS], next[RG_MAX_REPLICAS], rsnap[RG_MAX_REPLICAS];
  uint8_t rstate[RG_MAX_REPLICAS];
} rg_replica_view;

/* 64-byte message header, identical to the in-HBM slot layout. */
typedef struct rg_msg_view {
  uint8_t type, from, to, reject;
  uint32_t nent;
  uint64_t term, log_term, log_index, commit, hint, hint_high;
  uint32_t src_a, src_b; /* Propose: slab id, forward hop count */
} rg_msg_view;

typedef struct rg_entry_view {
  uint64_t term;
  uint32_t type, len, crc, bank;
} rg_entry_view;

typedef struct rg_tick_input {
  /* indexed by GLOBAL group g / replica g·replicas + slot, counted from this engine's first group
   * ranks·column_base; ranks·groups groups in all */
  const uint8_t* prop_target; /* [groups] slot receiving this tick's proposal batch, 0xFF none */
  const uint32_t* prop_count; /* [groups] entries in the batch (<= max_entries_per_msg) */
  const uint8_t* campaign;    /* [groups*replicas] nonzero: Peer.Campaign before the tick */
  const uint8_t* isolate;     /* [groups*replicas] nonzero: replica partitioned this tick */
  uint32_t flags;             /* RG_TICK_* */
  uint32_t _pad;
} rg_tick_input;

/* What the last tick moved, for the roofline numerator. Per SURVEY §8(d):
 * algorithmic_bytes = 128·replicas + 36·R·leaders + 128·msgs + (16+P)·repl_entries
 *                     + (12+P)·appended + P·leader_appended
 * bulk_bytes = the payload stage's share (bulk_kernel): every appended entry reads its payload
 * (sender ring or proposal slab) and writes payload + CRC; followers also read the sender's CRC:
 *   (2P+8)·appended − 4·leader_appended                                                   */
typedef struct rg_traffic {
  uint64_t replicas, leaders, msgs, repl_entries, appended, leader_appended;
  uint64_t algorithmic_bytes;
  uint64_t bulk_bytes;
} rg_traffic;

/* The committed-entry copy-back (rg_apply_committed / rg_apply_wait / rg_get_update): what dragonboat
 * hands to IOnDiskStateMachine.Update and raftd forwards as {"Index", "Cmd"} to POST /UpdateEntries
 * with headers raftd-node-id = shard, raftd-replica-id = replica (raft/state_machine.go:63-99,126-166),
 * shipped as RANGES: one rg_apply_run per run of consecutive entry indices of one replica, and per
 * entry only its Cmd's length and CRC (rg_apply_cmd, 8 B). Entry k of run r (0 <= k < r.count) is
 * Entry.Index r.first + k with length cmds[r.entry + k].len; its Cmd starts at payload + r.off +
 * the sum over the run's earlier entries of their lengths rounded up to 16 B (Cmds are packed back to
 * back, each rounded up to 16 B). A replica's runs come in index order, its entries contiguous in
 * cmds; a replica's window (processed at step start, processed] yields one run unless empty
 * entries (leader no-ops, config changes) split it. */
typedef struct rg_apply_run {
  uint64_t group;      /* global shard id (raftd-node-id) */
  uint32_t replica_id; /* raftd-replica-id: slot + 1 */
  uint32_t rid;        /* local replica id */
  uint64_t first;      /* statemachine.Entry.Index of the run's first entry */
  uint64_t entry;      /* its position in the rg_apply_cmd array */
  uint64_t off;        /* byte offset of its first Cmd in the payload buffer */
  uint32_t count;      /* entries in the run (>= 1) */
  uint32_t _pad;
} rg_apply_run;
typedef struct rg_apply_cmd {
  uint32_t len;        /* Cmd bytes */
  uint32_t crc;        /* CRC-32 of the Cmd as stored in the log */
} rg_apply_cmd;
typedef struct rg_apply_batch {
  const rg_apply_run* runs;
  uint64_t n_runs;
  const rg_apply_cmd* cmds;
  uint64_t n_entries;
  const uint8_t* payload;
  uint64_t payload_bytes;
} rg_apply_batch;

/* Persistence feed (rg_persist_collect, rg_get_update's persist section): dragonboat's
 * Update.EntriesToSave + pb.State + snapshot metadata, which it makes durable (LogDB SaveRaftState,
 * fsync) before a step's messages leave. Shipped as ranges: per replica one rg_persist_state; its
 * entries first..last follow as 8 B each (rg_persist_entry: length and CRC), their terms as runs
 * (rg_persist_term: term, count), their Cmds packed from payload + payload_off (each rounded up to
 * 16 B). Entry k of a replica is index first + k, at entries[entry_off + k]. */
typedef struct rg_persist_state {
  uint64_t group;       /* global shard id */
  uint32_t replica_id;  /* slot + 1 */
  uint32_t rid;         /* local replica id */
  uint64_t term, vote, commit;                                 /* pb.State */
  uint64_t last, marker, marker_term, snap_index, snap_term;   /* log end, compaction / snapshot */
  uint64_t first;       /* entries first..last follow (none if first > last); the log keeps its
                           entries below first, drops those above last and at or below marker */
  uint64_t entry_off;   /* position of this replica's first entry in the entries array */
  uint32_t members, snap_members; /* voting membership now and at the snapshot */
  uint64_t payload_off; /* byte offset of its first Cmd in the payload */
  uint64_t term_off;    /* its first term run in the terms array */
  uint32_t n_terms;     /* its term runs (their counts add up to last - first + 1) */
  uint32_t _pad;
} rg_persist_state;

#define RG_PERSIST_CONFIG 0x80000000u /* rg_persist_entry.len: a ConfigChange (the low bits: its descriptor) */
typedef struct rg_persist_entry {
  uint32_t len;         /* an application entry's Cmd bytes, or RG_PERSIST_CONFIG | descriptor */
  uint32_t crc;         /* CRC-32 of the Cmd (0 for none) */
} rg_persist_entry;
typedef struct rg_persist_term {
  uint64_t term;
  uint64_t count;       /* consecutive entries at this term */
} rg_persist_term;
typedef struct rg_persist_batch {
  const rg_persist_state* states;
  uint64_t n_states;
  const rg_persist_entry* entries;
  uint64_t n_entries;
  const rg_persist_term* terms;
  uint64_t n_terms;
  const uint8_t* payload;
  uint64_t payload_bytes;
} rg_persist_batch;

/* Snapshot events of the last tick (rg_snapshot_events): where dragonboat's rsm calls the state
 * machine's RecoverFromSnapshot (an InstallSnapshot restored the replica's log) and
 * PrepareSnapshot + SaveSnapshot (SnapshotEntries applied since the last snapshot), which raftd
 * forwards to the application (raft/state_machine.go:186-275). Host order per replica and tick:
 * recover to `restored`, Update the tick's applied entries, then save the snapshot at `index`. */
#define RG_SNAP_TAKEN 1u    /* a snapshot at index/term was taken at the end of the tick */
#define RG_SNAP_RESTORED 2u /* the log was restored to a snapshot at `restored` during the tick */
typedef struct rg_snapshot_event {
  uint64_t group;       /* global shard id */
  uint32_t replica_id;  /* slot + 1 */
  uint32_t rid;         /* local replica id */
  uint32_t kind;        /* RG_SNAP_* bits */
  uint32_t _pad;
  uint64_t restored;    /* kind & RG_SNAP_RESTORED: snapshot index the log was restored to */
  uint64_t index, term; /* kind & RG_SNAP_TAKEN: the new snapshot's index (= applied) and term */
} rg_snapshot_event;

/* One proposal batch (rg_propose): `count` client commands handed to slot `slot` of shard `group`
 * (the node's local replica; a follower forwards them to its leader, a candidate drops them).
 * Cmd k of the batch is lens[first + k] bytes; the Cmds of a call are packed back to back in lens
 * order in its payload buffer (entry j starts at lens[0] + … + lens[j-1]). */
typedef struct rg_proposal {
  uint64_t group;  /* GLOBAL shard id */
  uint32_t slot;   /* replica slot (replica id - 1); must be hosted by this engine */
  uint32_t count;  /* 1 .. max_entries_per_msg */
  uint64_t first;  /* index of the batch's first Cmd in lens[] */
} rg_proposal;

/* ReadIndex (rg_read_index): replica `slot` of shard `group` asks for a linearizable read point
 * under a non-zero context (dragonboat's SystemCtx; the shim batches the tick's client reads of a
 * replica under one context). */
typedef struct rg_read_request {
  uint64_t group; /* GLOBAL shard id */
  uint32_t slot, _pad;
  uint64_t ctx;
} rg_read_request;
/* A read made ready (dragonboat's ReadyToRead): serve the reads of `ctx` — IOnDiskStateMachine.Lookup,
 * raftd's POST /Read (raft/state_machine.go:168-184) — once the replica has applied `index`. */
typedef struct rg_read_ready {
  uint64_t group;
  uint32_t replica_id, rid;
  uint64_t ctx, index;
} rg_read_ready;

typedef struct rg_engine rg_engine;

int rg_create(const rg_config* cfg, rg_engine** out);
void rg_destroy(rg_engine* e);
/* Every replica: becomeFollower(1) + bootstrap ConfigChange entries 1..R (AddNode for each initial
 * member), committed R; a join slot (rg_config.join_slots): becomeFollower(0), empty log. */
int rg_bootstrap(rg_engine* e);
/* Fill every proposal slab with the deterministic payload generator: the synthetic
 * Cmds (payload_bytes each) that tick-input proposals (rg_tick_input.prop_target) carry — the
 * benchmark's fast path. Client commands enter through rg_propose. */
int rg_fill_slabs(rg_engine* e);
/* Stage client commands for the next tick (its proposal step): n batches, Cmd bytes
 * in `payload` (host memory, copied before return; packed in lens order), lengths in `lens`
 * (each <= max_cmd_bytes; 0 = an empty Cmd, which commits but is not handed to Update). Calls before
 * one tick accumulate: batches for the same shard and slot are concatenated up to
 * max_entries_per_msg. All or nothing: RG_EINVAL (bad shard / slot / count / length, a slot hosted
 * elsewhere), RG_EFULL (a shard's batch would exceed max_entries_per_msg, or a second slot of one
 * shard in one tick) — nothing is staged then. The next rg_tick / rg_tick_device takes the staged
 * batches and must not also carry rg_tick_input.prop_target. */
int rg_propose(rg_engine* e, const rg_proposal* props, size_t n, const uint8_t* payload, const uint32_t* lens);
/* Register a long-lived host buffer the caller stages Cmds in (hipHostRegister: page-locked until
 * rg_host_unregister or rg_destroy). An rg_propose whose payload lies inside a registered range and
 * whose Cmds are packed the way the device arena holds them (every Cmd of a batch but its last a
 * multiple of 16 B, the batches in few contiguous runs) is copied by DMA straight from it, without
 * the host copy into pinned staging (DESIGN.md §4 "Ingest"); still copied before return. Ranges may
 * not overlap. */
int rg_host_register(rg_engine* e, const void* p, size_t bytes);
int rg_host_unregister(rg_engine* e, const void* p);
/* One tick for every replica. Input arrays are host pointers (copied before launch; NULL =
 * none). Synchronous with respect to the host buffers, asynchronous on the device. */
int rg_tick(rg_engine* e, const rg_tick_input* in);
/* Same, with the input arrays already resident in device memory (no copies). */
int rg_tick_device(rg_engine* e, const rg_tick_input* in);
/* k ticks with the same device-resident inputs (the steady-state pattern of a batch driver): without
 * flags, k rg_tick_device calls; with RG_TICKN_GRAPH, one captured HIP graph of the k ticks, replayed
 * with one launch (the parameter blocks are written into the graph's pinned slots before each
 * replay, so results equal k rg_tick_device calls bit for bit). The graph needs a one-rank engine
 * (ranks 1, wire_all 0), nothing staged by rg_propose / rg_read_index / rg_config_change, timing off,
 * and k a multiple of lcm(2, num_slabs), at most 64 (slabs rg_propose wrote get the generator's Cmds
 * back first, as a tick-input batch would; the last tick's slab must not be one); it is captured
 * on first use and again whenever k, the inputs, the stream or the parity of the tick count change. */
#define RG_TICKN_GRAPH 1u
/* RG_TICKN_RESIDENT (metadata-only engines, payload_bytes 0, one rank, replicas <= 4): the k ticks
 * in ONE launch of a resident control kernel — a workgroup holds every replica of 64 groups, so a
 * tick's messages stay inside it, and a workgroup barrier replaces the kernel boundary between
 * ticks. Same results as k rg_tick_device calls; k <= 64; the other conditions as for a graph. */
#define RG_TICKN_RESIDENT 2u
int rg_tick_device_n(rg_engine* e, const rg_tick_input* in, uint32_t k, uint32_t flags);
/* Launch work on this HIP stream (hipStream_t) instead of the engine's own. */
int rg_set_stream(rg_engine* e, void* stream);
/* Make the engine's stream wait, on the device, for every launched tick to finish (a tick's
 * payload stage runs on a second internal stream); no host synchronisation. */
int rg_join(rg_engine* e);
/* rg_join, then block the host until the engine's stream is idle. */
int rg_sync(rg_engine* e);
/* Per-launch kernel timing with HIP events on the streams the kernels run on (measurement
 * only). enable=1 times both kernels (four event records per tick), enable=2 bulk_kernel only
 * (two), 0 stops; a non-zero value zeroes the totals. enable | (n << 8): only every n-th tick
 * (tick count divisible by n) is timed — each timed event record costs its tick tens of µs. */
int rg_timing(rg_engine* e, int enable);
/* Synchronises, then returns the summed durations (ms) and launch counts since rg_timing(e, 1):
 * index 0 = control_kernel, 1 = bulk_kernel. */
int rg_kernel_ms(rg_engine* e, double* ms /*[2]*/, uint64_t* launches /*[2]*/);
/* Measurement across engines (column halves on their own streams): rg_timing_epoch records one
 * process-wide reference event on `device` (and waits for it); from then on every timed launch of
 * every engine on that device is also kept as {tick, start, end} in ms after the epoch, so launches
 * on different streams can be laid on one timeline (the span of overlapping launches, not the sum
 * of their durations). rg_kernel_events returns up to cap of the kernel's (0 control, 1 bulk)
 * launches since rg_timing(e, on); *n = how many there are. Synchronises like rg_kernel_ms. */
int rg_timing_epoch(int device);
int rg_kernel_events(rg_engine* e, int kernel, uint64_t* ticks, double* start_ms, double* end_ms, uint64_t cap,
                     uint64_t* n);
uint64_t rg_tick_count(const rg_engine* e);

int rg_read_replicas(rg_engine* e, uint32_t first_rid, uint32_t n, rg_replica_view* out);
/* Messages `rid` emitted to slot `dst` in the last tick; returns the count, fills up to cap
 * headers and, if terms != NULL, cap * max_entries_per_msg inline entry terms (bank bit
 * cleared). */
int rg_read_msgs(rg_engine* e, uint32_t rid, uint32_t dst, rg_msg_view* out, uint32_t cap, uint64_t* terms);
/* Log entries first_index .. first_index+n-1 of replica rid (must lie in (marker, last]); payload (if
 * not NULL, at most n * max_cmd_bytes bytes are written): the Cmds of the application entries, packed
 * back to back in entry order at their own lengths (out[k].len bytes each; entries with an empty Cmd
 * and ConfigChange entries take none). */
int rg_read_entries(rg_engine* e, uint32_t rid, uint64_t first_index, uint32_t n, rg_entry_view* out,
                    uint8_t* payload);
/* Replace replica rid's state and its log (marker, last]: terms[k] (< 2^36), types[k] (RG_ENTRY_*,
 * | RG_ENTRY_EMPTY), payloads = the Cmds packed back to back in entry order: an application entry that
 * is not RG_ENTRY_EMPTY takes lens[k] bytes (lens NULL: payload_bytes), any other entry none; a
 * ConfigChange entry's lens[k] is its descriptor. The replica's Cmds move to a fresh payload stream
 * (RG_ENOMEM: the page pool is empty; RG_EFULL: longer than stream_pages). Not for a replica whose
 * messages of the last tick are still to be delivered. */
int rg_import_replica(rg_engine* e, uint32_t rid, const rg_replica_view* v, const uint64_t* terms,
                      const uint32_t* types, const uint8_t* payloads, const uint32_t* lens);
/* Enqueue a message as if `rid_src` had emitted it in the last tick (delivered next tick). */
int rg_deliver(rg_engine* e, uint32_t rid_src, const rg_msg_view* m);
/* NodeHost.GetLeaderID for GLOBAL group `group`, as this engine's replicas of it know it: a local
 * replica that leads at the highest local term, else that replica's known leader. */
int rg_leader(rg_engine* e, uint32_t group, uint64_t* leader_id, uint64_t* term, int* valid);
/* Sum over groups of the highest committed index among the group's replicas (ranks > 1: over
 * the slot-0 replicas this engine hosts, so the sum over ranks counts every group once). */
int rg_sum_committed(rg_engine* e, uint64_t* out);
/* Message / entry counts of the last tick and the algorithmic bytes they imply. */
int rg_last_tick_traffic(rg_engine* e, rg_traffic* out);
/* ---- Inter-rank exchange (ranks > 1 or wire_all): the transport plug (dragonboat ITransport's
 * place). Messages a replica emitted in the last tick to a replica on another rank travel as one
 * region per destination rank; the caller moves the regions (RCCL all-to-all over xGMI, or any
 * transport) between rg_tick calls:
 *   rg_wire_plan(e, send_bytes)        sizes of this rank's outbound regions (synchronises)
 *   rg_wire_pack(e, buf, cap)          writes region r at offset send_bytes[0] + … + send_bytes[r-1]
 *                                      of the device buffer buf (async, on the engine's stream)
 *   transport                          region r of rank a → rank r; each rank learns recv_bytes
 *   rg_wire_recv(e, buf, recv_bytes)   regions from every rank, concatenated in rank order in the
 *                                      device buffer buf, are unpacked for the next tick (async);
 *                                      buf must stay valid until that tick has completed on the
 *                                      device (followers read payloads straight out of it).
 * rg_tick fails with RG_EINVAL if a tick after the first runs without rg_wire_recv.
 * Two ways to size the regions:
 *   rg_wire_plan        exact: waits for the plan kernel and returns the bytes each region needs;
 *                       the transport then has to tell each rank what it receives (a size exchange).
 *   rg_wire_plan_fixed  fixed capacity: send_bytes / recv_bytes are capacities both ends of every
 *                       link already agree on (a rule over numbers both see), so one
 *                       all-to-all per tick moves the regions and nothing waits for the tick that
 *                       made the messages. The rule reads the needs of the exchange two before this
 *                       one: a bounded wait (an event two exchanges old; the host runs at most two
 *                       exchanges ahead of the device). A unit (one replica pair's messages) that does
 *                       not fit its region is dropped whole — the messages are lost in transit, which
 *                       Raft tolerates — and counted (rg_wire_dropped). Capacities start at the most a
 *                       steady tick can need (a full Replicate plus one header per unit, or the worst
 *                       case of K messages when smaller; a link whose worst case fits never drops),
 *                       then follow the largest need of the last 8 exchanges (+1/16): up at once past
 *                       a need that overflowed, down by at most 1/8 per exchange. A region header whose
 *                       need is impossible for its link fails the call (RG_EINVARIANT). */
int rg_wire_plan(rg_engine* e, uint64_t* send_bytes /*[ranks]*/);
int rg_wire_plan_fixed(rg_engine* e, uint64_t* send_bytes /*[ranks]*/, uint64_t* recv_bytes /*[ranks]*/);
int rg_wire_pack(rg_engine* e, void* send_buf, uint64_t send_cap);
/* rg_wire_pack with the caller's layout: region r at base + region_off[r] (16-B aligned, inside
 * base_cap, regions not overlapping). The region to this rank itself can be packed straight into
 * the place where rg_wire_recv will read it (its receive buffer at that region's offset), so the
 * transport moves nothing for it — what rg_wire_exchange does. */
int rg_wire_pack_at(rg_engine* e, void* base, const uint64_t* region_off /*[ranks]*/, uint64_t base_cap);
int rg_wire_recv(rg_engine* e, const void* recv_buf, const uint64_t* recv_bytes /*[ranks]*/);
/* Messages dropped so far because their unit did not fit a fixed-capacity region. */
int rg_wire_dropped(rg_engine* e, uint64_t* msgs);
/* The whole exchange in one call: plan, pack into an engine-owned send buffer, t->alltoallv into an
 * engine-owned receive buffer, and rg_wire_recv. Sizing: rg_wire_plan_fixed — the tick's one
 * collective, no host sync, no size exchange — unless rg_config.wire_exact is set and the transport has
 * allgather_u64: then rg_wire_plan, and the sizes go through t->allgather_u64 first. Every rank of the
 * cluster calls it between the same two ticks (all with the same sizing). A host in any
 * language gets multi-GPU replication from this call plus a transport: the built-in RCCL one
 * (rg_rccl_open) or its own.
 * *sent_bytes (if not NULL) = the bytes this rank sent to other ranks. The transport's callbacks return 0 on success. alltoallv gets device buffers and the engine's
 * HIP stream. Its transfers must come after the work already on `stream` (the pack), and the
 * work enqueued on `stream` after it returns (the unpack) must come after its transfers. It can
 * enqueue on `stream` itself, order a stream of its own by events both ways (the RCCL transport),
 * or synchronise `stream` and complete before returning (a host-staged transport). Region r of `send`
 * (send + soff[r], ssize[r] bytes) goes to rank r; region r of `recv`
 * (recv + roff[r], rsize[r] bytes) comes from rank r. allgather_u64 (used by the exact sizing; may be
 * NULL, which makes the sizing fixed) is a host-memory, blocking all-gather of n values per rank:
 * all[r * n + i] = value i of rank r. */
typedef struct rg_transport {
  void* user;
  int (*allgather_u64)(void* user, const uint64_t* mine, uint64_t* all, uint32_t n);
  int (*alltoallv)(void* user, const void* send, const uint64_t* soff, const uint64_t* ssize, void* recv,
                   const uint64_t* roff, const uint64_t* rsize, void* stream);
} rg_transport;
int rg_wire_exchange(rg_engine* e, const rg_transport* t, uint64_t* sent_bytes /* nullable: bytes to other ranks */);
/* Built-in RCCL transport (librccl loaded at run time; the one a PyTorch process already holds
 * is reused). Rank 0 calls rg_rccl_unique_id and hands the 128 bytes to every rank out of band
 * (raftd: over its own control channel); each rank then calls rg_rccl_open with its device.
 * Each peer region moves in pieces of at most 256 MiB ("The 1 GiB contract").
 * rg_rccl_close destroys the communicator. */
int rg_rccl_unique_id(uint8_t id[128]);
int rg_rccl_open(const uint8_t id[128], int32_t nranks, int32_t rank, int32_t device, rg_transport* out);
int rg_rccl_close(rg_transport* t);
/* Committed-entry copy-back: the non-empty application entries that the
 * replicas whose slot bit is set in slot_mask applied in the last tick — config changes, leader
 * no-ops and snapshot-restored ranges excluded, as dragonboat's rsm does before Update — grouped
 * by replica in device order (slot by slot, shards ascending within a slot), each replica's
 * entries in index order, as runs (rg_apply_run / rg_apply_cmd above). Compacted on the device, then
 * copied back by one hipMemcpyAsync into engine-owned pinned memory: *out points into it, valid until
 * the next rg_apply_committed; only run heads, 8 B per entry and the Cmd bytes cross PCIe.
 * Synchronous. */
int rg_apply_committed(rg_engine* e, uint32_t slot_mask, rg_apply_batch* out);
/* Asynchronous, double-buffered copy-back (the same batch as rg_apply_committed) into engine-owned
 * pinned buffer `buf` (0 or 1). On the engine's stream right after the tick (before a later tick can
 * reuse the window's log slots and pages): the count and scan kernels, then ONE host synchronisation
 * for the batch's size (the buffers grow when it exceeds them), then the gather kernel into device
 * staging. The D2H leg then runs on the engine's copy stream — a copy kernel of a few workgroups
 * streaming into host-mapped memory (default), or an SDMA engine (RAFTGPU_APPLY_SDMA=1, the only
 * runtime hook of the copy-back; the runtime's hipMemcpyAsync is the -DRG_AB_APPLY_MEMCPY build
 * variant) — so the caller may issue the
 * next tick before it completes. Whether that overlap pays depends on the platform (DESIGN.md §7,
 * INTEGRATION.md "Copy-back schedule"). */
int rg_apply_async(rg_engine* e, uint32_t slot_mask, int buf);
/* Wait for buffer `buf`'s gather; *out points into engine-owned pinned memory, valid until the next
 * rg_apply_async into `buf`. */
int rg_apply_wait(rg_engine* e, int buf, rg_apply_batch* out);
/* Host WAL feed: for every replica whose log or hard state changed in the last
 * tick (full != 0, or no tick yet: every replica, whole log window), one rg_persist_state and the
 * entries it rewrote as ranges (rg_persist_batch above), gathered on the device and copied back by one
 * hipMemcpyAsync into engine-owned pinned memory (*out points into it, valid until the next call).
 * Make them durable before the next tick delivers the last tick's messages. Synchronous. Restart =
 * rg_import_replica of the replayed state. */
int rg_persist_collect(rg_engine* e, int full, rg_persist_batch* out);
/* Snapshot events of the last tick for replicas whose slot bit is set in slot_mask, one per
 * replica in device order (slot by slot, shards ascending within a slot), compacted on the device and copied back by one hipMemcpyAsync. *n = the count;
 * if *n > cap nothing is copied and RG_EFULL is returned. Synchronous. */
int rg_snapshot_events(rg_engine* e, uint32_t slot_mask, rg_snapshot_event* events, uint64_t cap, uint64_t* n);
/* ---- One hand-off per tick (dragonboat Peer.GetUpdate / Peer.Commit): everything the
 * host must act on after a tick, gathered on the device in one pass — the persistence feed
 * (rg_persist_collect), the committed entries for IOnDiskStateMachine.Update (rg_apply_committed),
 * the snapshot events (rg_snapshot_events) and the reads made ready (rg_read_index_results) — with
 * one host synchronisation for the counts and one D2H copy of all sections. The pointers are
 * engine-owned pinned memory, valid until the next rg_get_update or rg_destroy. slot_mask selects
 * the replicas every section reports (the node's slots): their persistence records (those whose log
 * or hard state changed; all of them with their whole log window under RG_UPDATE_FULL_STATE: a
 * checkpoint), committed entries, snapshot events and reads. Sections not asked for are empty. */
#define RG_UPDATE_PERSIST 1u     /* EntriesToSave + State (rg_persist_collect) */
#define RG_UPDATE_COMMITTED 2u   /* CommittedEntries for Update (rg_apply_committed) */
#define RG_UPDATE_SNAPSHOTS 4u   /* snapshot events (rg_snapshot_events) */
#define RG_UPDATE_READS 8u       /* ReadyToReads (rg_read_index_results) */
#define RG_UPDATE_ALL 15u
#define RG_UPDATE_FULL_STATE 16u /* persistence section: every replica, whole log window */
/* With RG_UPDATE_PERSIST and RG_UPDATE_COMMITTED together the committed section is BY REFERENCE:
 * runs and {len, crc} only, committed.payload = NULL and payload_bytes = 0. Every committed entry's Cmd
 * was delivered in this or an earlier persist section of the same replicas (a replica commits only
 * what it has in its log, and its log writes are persisted in the update of the tick that made them);
 * the host keeps persisted Cmds until the replica has applied them — dragonboat hands Update its
 * entries from its own in-memory log the same way. Entry k of a run is its replica's persisted entry
 * r.first + k; r.off is where its Cmd would sit in a packed payload. Each Cmd then crosses PCIe once
 * per hand-off stream. Entries of rg_import_replica never pass through a persist section: a host that
 * imports keeps their Cmds itself (it read them from its WAL). RG_UPDATE_COMMITTED_CMDS ships the Cmds
 * anyway (and rg_apply_committed / rg_apply_async always do). */
#define RG_UPDATE_COMMITTED_CMDS 32u
typedef struct rg_update {
  uint64_t tick;                          /* ticks run when the update was taken */
  rg_persist_batch persist;               /* states, entries, term runs, Cmds (rg_persist_batch) */
  rg_apply_batch committed;               /* the committed entries, as runs (rg_apply_run) */
  const rg_snapshot_event* snapshots;
  uint64_t n_snapshots;
  const rg_read_ready* reads;
  uint64_t n_reads;
  uint32_t slot_mask, flags;
} rg_update;
int rg_get_update(rg_engine* e, uint32_t slot_mask, uint32_t flags, rg_update* out);
/* Peer.Commit for an update the host has made durable and handed to the state machine: with
 * RG_COMMIT_APPLIED, every replica of u->slot_mask reports applied = its processed index
 * (NotifyRaftLastApplied; meaningful with rg_config.apply_feedback = 1). The update's buffers may
 * be reused afterwards. */
#define RG_COMMIT_APPLIED 1u
int rg_commit_update(rg_engine* e, const rg_update* u, uint32_t flags);
/* Stage ReadIndex requests for the next tick (dragonboat's NodeHost.ReadIndex → Peer.ReadIndex): a
 * leader that has committed an entry in its term records its commit index and confirms leadership
 * with one heartbeat round carrying the context; a follower forwards the request to its leader,
 * which answers with a ReadIndexResp once confirmed. A leader keeps up to RG_READ_QUEUE requests
 * pending in arrival order (dragonboat's readIndex queue; a context already pending is not added
 * twice, one more is dropped and counted in drops — the shim retries): when a quorum has confirmed
 * one, it and every request queued before it become ready at its index, and every regular
 * heartbeat carries the newest pending context. RG_EINVAL: bad shard / slot, ctx 0, or a replica
 * hosted by another rank (nothing staged). A later request for the same replica in the same tick
 * replaces the earlier one. */
#define RG_READ_QUEUE 4
int rg_read_index(rg_engine* e, const rg_read_request* reqs, size_t n);
/* Reads made ready in the last tick for replicas whose slot bit is set — up to RG_READ_QUEUE per
 * replica, in the order they became ready (more in one tick are dropped, counted) — replicas in
 * device order; compacted on the device, one hipMemcpyAsync. *n = count; RG_EFULL if > cap. */
int rg_read_index_results(rg_engine* e, uint32_t slot_mask, rg_read_ready* out, uint64_t cap, uint64_t* n);
/* Stage a membership change for the next tick: NodeHost.SyncRequestAddReplica (op RG_CC_ADD) /
 * SyncRequestDeleteReplica (RG_CC_REMOVE) of slot `target` of global shard `group`
 * (raft/raft_manager.go:165-185), proposed at the local replica `slot` after that tick's Cmd batch.
 * The leader appends one ConfigChange entry (a follower forwards it; a second change while one is
 * in flight becomes an empty entry and counts a drop); every replica applies it when the entry is
 * handed to its state machine: quorum, elections, replication and snapshots then follow the new
 * membership. RG_EINVAL: bad shard / slot / target / op, or a replica hosted by
 * another rank; RG_EFULL: a change is already staged for the shard this tick. */
#define RG_CC_ADD 1u
#define RG_CC_REMOVE 2u
int rg_config_change(rg_engine* e, uint64_t group, uint32_t slot, uint32_t op, uint32_t target);
/* Peer.NotifyRaftLastApplied for n local replicas: replica rids[k]'s state machine has applied
 * through index[k] (<= its processed index — config changes and empty entries included, which the
 * state machine never sees). With rg_config.apply_feedback = 1 this is how `applied` moves: it gates
 * campaigns (hasConfigChangeToApply: committed > applied) and snapshots (SnapshotEntries applied
 * since the last one). RG_EINVAL (nothing changed) if an index exceeds processed or a rid is bad. */
int rg_notify_applied(rg_engine* e, const uint32_t* rids, const uint64_t* index, size_t n);
/* Log compaction for GLOBAL shard `group` between ticks (SURVEY §8b rg_compact; raftd compacts only on
 * its SnapshotEntries / CompactionOverhead schedule, raft/raft_manager.go:97-98, which the engine runs by
 * itself — this is the explicit form): every replica of the shard hosted here compacts its log to
 * min(index, its latest snapshot index) when that is above its marker, exactly as a snapshot's
 * compaction does (entries at or below it are gone; a follower that needs them gets InstallSnapshot);
 * the payload stream below is released by the next tick. *compacted (nullable) = replicas compacted.
 * RG_EINVAL for a shard outside this engine. Synchronises. */
int rg_compact(rg_engine* e, uint64_t group, uint64_t index, uint32_t* compacted);
/* Whole-table digest of this engine's replicas: out[0] = the sum over replicas of an
 * fmix64 chain over the replica's rg_replica_view fields (remotes of slots < replicas), out[1] = the
 * sum of a chain over its log entries (marker, last] (term, then type | len << 8 | crc << 32), each
 * chain seeded by the global replica id. Order-independent, so the digests of several ranks add up to
 * the cluster's; the oracle's or_digest is the same function — a parity check of every replica and
 * every log entry at any size, in one pass on the device. */
int rg_digest(rg_engine* e, uint64_t* out /*[2]*/);
/* Global group and global replica id (group·replicas + slot) of local replica rid. */
int rg_global_id(rg_engine* e, uint32_t rid, uint64_t* group, uint64_t* global_rid);
/* Measurement helper: this device's streaming-copy bandwidth, (read + write bytes) / s, of a
 * 16-B-per-lane non-temporal grid-stride copy of `bytes` (the bulk kernel's access shape), best
 * of `reps` launches timed with HIP events. Allocates and frees 2 x bytes. */
int rg_probe_copy(int32_t device, uint64_t bytes, int32_t reps, double* gbps);
/* Device bytes held by the engine. */
uint64_t rg_device_bytes(const rg_engine* e);
/* The payload page pool: pages in all, pages free (after the last launch), and
 * whether an allocation ever found it empty (the engine is then poisoned: RG_ERR_POOL). Synchronises. */
int rg_pool_stats(rg_engine* e, uint64_t* total_pages, uint64_t* free_pages, int* failed);
const char* rg_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
