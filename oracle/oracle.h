/*
 * oracle.h — CPU restatement of dragonboat v4's per-shard Raft step (TEST INFRASTRUCTURE).
 *
 * This is the parity oracle for raftd-amd's HIP step engine. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. It is never a
 * fallback for the product path.
 *
 * PARITY UNPINNED against dragonboat: the algorithm lives in the third-party Go module
 * github.com/lni/dragonboat/v4 v4.0.0-20240618143154-6a1623140f27 (/root/reference/go.mod:9,
 * go.sum:268-269), package internal/raft, which is not present in this container and cannot
 * be built here (no Go toolchain). This file restates it from SURVEY.md Appendix A with the
 * VERIFY decisions recorded in DESIGN.md §1. It is cross-checked against the independent
 * Python restatement oracle/pyraft.py and the known-answer tests in tests/golden/.
 * Call sites in the reference that reach this path: raft/raft_manager.go:92-100 (config),
 * :109 (NewNodeHost), :142 (StartOnDiskReplica), raft/members.go:21 (GetLeaderID).
 */
#ifndef RAFT_ORACLE_H
#define RAFT_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_MAX_R 8
#define OR_RQ 4 /* ReadIndex requests a leader holds pending, and reads a replica makes ready per step */
#define OR_MAX_CMD (1u << 24) /* the longest Cmd max_cmd_bytes may name (16 MiB; the engine's MAX_CMD) */

/* raftpb.MessageType numbering as recalled (VERIFY); only the values below are used. */
enum {
  OR_LOCAL_TICK = 0, OR_ELECTION = 1, OR_LEADER_HEARTBEAT = 2, OR_NOOP = 4, OR_PROPOSE = 7,
  OR_CHECK_QUORUM = 10, OR_REPLICATE = 12, OR_REPLICATE_RESP = 13, OR_REQUEST_VOTE = 14,
  OR_REQUEST_VOTE_RESP = 15, OR_INSTALL_SNAPSHOT = 16, OR_HEARTBEAT = 17, OR_HEARTBEAT_RESP = 18,
  OR_READ_INDEX = 19, OR_READ_INDEX_RESP = 20
};
enum { OR_FOLLOWER = 0, OR_CANDIDATE = 1, OR_LEADER = 2 };
enum { OR_RETRY = 0, OR_WAIT = 1, OR_REPLICATE_ST = 2, OR_SNAPSHOT = 3 };
enum { OR_ENTRY_APP = 0, OR_ENTRY_CONFIG = 1 };
/* A ConfigChange entry's descriptor, kept in its `len` field (it has no Cmd): op << 4 | (slot + 1);
 * 0 = the bootstrap entries, which change nothing */
enum { OR_CC_ADD = 1, OR_CC_REMOVE = 2 };
#define OR_CC(op, slot) ((uint32_t)(op) << 4 | ((uint32_t)(slot) + 1u))
#define OR_ENTRY_EMPTY 0x100u /* import: application entry with an empty Cmd (no payload) */
enum {
  OR_ERR_CONFLICT_COMMITTED = 1, OR_ERR_COMMIT_BEYOND_LAST = 2, OR_ERR_RING_FULL = 4,
  OR_ERR_CRC = 8, OR_ERR_EMPTY_SNAPSHOT = 16,
  OR_ERR_TERM_LIMIT = 128 /* a campaign at term 2^36 - 1 (the ring word's term field) was refused */
};
#define OR_TERM_MAX ((1ull << 36) - 1) /* terms are 36-bit (the GPU ring word's term field) */
#define OR_TICK_NO_LOCALTICK 1u

typedef struct or_config {
  uint32_t groups, replicas, log_capacity, payload_bytes;
  uint32_t max_entries_per_msg, max_msgs_per_pair, num_slabs;
  uint32_t election_rtt, heartbeat_rtt, check_quorum;
  uint32_t snapshot_entries, compaction_overhead;
  uint32_t drop_ppm;
  uint32_t group_base; /* global id of group 0: an oracle of a window of groups [base, base+groups)
                          reproduces that window of a larger run (groups are independent; RNG keys,
                          loss hashes and payloads use the global id; tick inputs are the window's) */
  uint64_t seed;
  uint32_t crc32c; /* entry checksum: 0 = CRC-32/IEEE (zlib), 1 = CRC-32C (Castagnoli) */
  uint32_t apply_feedback; /* 0: applied follows processed at the end of every step (the state machine
                              keeps up); 1: applied moves only by or_notify_applied (NotifyRaftLastApplied) */
  uint32_t initial_members; /* bootstrap membership, bit s = slot s (StartOnDiskReplica's initialMembers);
                               0 = every slot */
  uint32_t max_cmd_bytes;   /* longest Cmd (payload_bytes .. OR_MAX_CMD; 0 = payload_bytes) */
  uint32_t stream_pages;    /* the stream capacity rule's window, 4-KiB pages (power of two; 0 = as
                               rg_create sizes it) */
  uint32_t join_slots;      /* slots started with join = true: empty log, term 0, no membership */
  uint32_t _pad;
} or_config;

/* Field order identical to rg_replica_view (include/raftgpu.h) so tests compare by name. */
typedef struct or_replica_view {
  uint64_t term, vote, leader, committed, applied, last, marker, marker_term;
  uint64_t snap_index, snap_term, cap_base, processed;
  uint32_t role, election_tick, heartbeat_tick, rand_timeout, rng_ctr;
  uint32_t granted, responded, active, err, drops;
  uint32_t members;      /* voting membership as this replica applied it, bit s = slot s */
  uint32_t snap_members; /* the membership its latest snapshot records */
  uint32_t cc_pending;   /* leader: a config change is in flight (pendingConfigChange) */
  uint32_t _mpad;
  uint64_t match[OR_MAX_R], next[OR_MAX_R], rsnap[OR_MAX_R];
  uint8_t rstate[OR_MAX_R];
} or_replica_view;

typedef struct or_msg_view {
  uint8_t type, from, to, reject;
  uint32_t nent;
  uint64_t term, log_term, log_index, commit, hint, hint_high;
  uint32_t src_a, src_b; /* Propose: slab id, hop count */
} or_msg_view;
/* A Propose message carries its nent entries (Cmd bytes + length, like pb.Message.Entries of a
 * forwarded MsgProp); its header `hint` is the mask of entries with a non-empty Cmd (bit k). */

/* One proposal batch handed to a shard's replica (NodeHost.Propose → Peer.ProposeEntries):
 * `count` Cmds whose lengths are lens[first .. first+count) and whose bytes are packed back to back
 * in lens order in the payload buffer of or_propose. */
typedef struct or_proposal {
  uint64_t group;  /* global shard id (group_base + window-local id) */
  uint32_t slot;   /* replica slot the node hands the batch to */
  uint32_t count;  /* entries, 1 .. max_entries_per_msg */
  uint64_t first;  /* its first entry in lens[] */
} or_proposal;

typedef struct or_entry_view {
  uint64_t term;
  uint32_t type, len, crc, _pad;
} or_entry_view;

typedef struct or_tick_input {
  const uint8_t* prop_target; /* [G] slot, 0xFF none; NULL = no proposals */
  const uint32_t* prop_count; /* [G] */
  const uint8_t* campaign;    /* [G*R] nonzero → Handle(Election) before LocalTick; NULL none */
  const uint8_t* isolate;     /* [G*R] nonzero → all messages to/from the replica lost */
  uint32_t flags;
} or_tick_input;

typedef struct or_engine or_engine;

int or_create(const or_config* cfg, or_engine** out);
void or_destroy(or_engine* e);
int or_bootstrap(or_engine* e);
/* One tick over all groups using `nthreads` worker threads (group g → worker g % nthreads,
 * dragonboat's step-worker partition). */
int or_tick(or_engine* e, const or_tick_input* in, int nthreads);
uint64_t or_tick_count(const or_engine* e);

int or_get_replica(const or_engine* e, uint32_t rid, or_replica_view* out);
/* Views of replicas first .. first+n-1 (bulk comparisons at full size). */
int or_get_replicas(const or_engine* e, uint32_t first, uint32_t n, or_replica_view* out);
/* Messages emitted by `rid` to slot `dst` in the last tick. Returns count; fills up to cap. */
int or_get_msgs(const or_engine* e, uint32_t rid, uint32_t dst, or_msg_view* out, uint32_t cap);
/* Inline entry terms of message k (rid → dst). */
int or_get_msg_terms(const or_engine* e, uint32_t rid, uint32_t dst, uint32_t k, uint64_t* terms, uint32_t cap);
/* Log entry at `index` of replica rid (must be in (marker, last]). payload may be NULL (else len bytes). */
int or_get_entry(const or_engine* e, uint32_t rid, uint64_t index, or_entry_view* out, uint8_t* payload);
/* Replace a replica's state and log (entries for indices marker+1 .. last). payloads: the Cmds packed
 * back to back in entry order; an application entry that is not OR_ENTRY_EMPTY takes lens[k] bytes
 * (lens NULL: payload_bytes), any other none (a ConfigChange's lens[k] is its descriptor). Its
 * payload stream restarts at position 0 (as rg_import_replica's). */
int or_import_replica(or_engine* e, uint32_t rid, const or_replica_view* v,
                      const uint64_t* terms, const uint32_t* types, const uint8_t* payloads,
                      const uint32_t* lens);
/* Stage caller proposals for the next tick (its step 4 instead of tick-input prop_target; a tick
 * given both fails). Batches for the same group and slot are concatenated (at most
 * max_entries_per_msg in all); a second slot of one group in one tick, an empty or oversized batch,
 * a Cmd longer than payload_bytes or a group outside the window fail the whole call, staging
 * nothing: -1 invalid, -3 batch full. Cmd bytes packed in lens order (entry j at the sum of
 * lens[0..j)). */
int or_propose(or_engine* e, const or_proposal* p, size_t n, const uint8_t* payload, const uint32_t* lens);
/* Stage a membership change for the next tick (SyncRequestAddReplica / SyncRequestDeleteReplica,
 * raft/raft_manager.go:165-185): a ConfigChange entry adding (OR_CC_ADD) or removing (OR_CC_REMOVE)
 * slot `target`, proposed at replica `slot` of shard `group` after that tick's Cmd batch. -1 invalid,
 * -3 a change is already staged for the shard this tick. */
int or_config_change(or_engine* e, uint64_t group, uint32_t slot, uint32_t op, uint32_t target);
/* rg_compact: between ticks, compact the log of every replica of global shard `group`
 * to min(index, its snap_index) when that is above its marker (marker_term = the term there); the
 * payload stream below it is released by the next tick, as after a snapshot's compaction. Returns the
 * number of replicas compacted, or -1 for a shard outside the engine. */
int or_compact(or_engine* e, uint64_t group, uint64_t index);
/* Append a message to rid_src's most recent outbox so it is delivered next tick. Replicate
 * entries are taken from the sender's current log (indices log_index+1 ..). */
int or_deliver(or_engine* e, uint32_t rid_src, const or_msg_view* m);
/* Non-empty application entries replica rid applied in the last step (IOnDiskStateMachine.Update
 * input), in index order. Returns the count; fills up to cap (payload: their Cmds packed back to back
 * at their own lengths). Any output may be NULL. */
int or_get_applied(const or_engine* e, uint32_t rid, uint64_t* index, or_entry_view* out, uint8_t* payload,
                   uint32_t cap);
/* Peer.NotifyRaftLastApplied: the state machine of replica rid has applied through `index`
 * (<= processed, else -1). With apply_feedback = 1 this is the only way `applied` moves (besides a
 * restored snapshot); it gates campaigns (hasConfigChangeToApply) and snapshots. */
int or_notify_applied(or_engine* e, uint32_t rid, uint64_t index);
/* ReadIndex (dragonboat's ReadIndex protocol, Raft thesis §6.4) for the next tick: replica `slot` of
 * shard `group` asks for a linearizable read point under context ctx (non-zero). At most one request
 * per replica per tick (a later one replaces an earlier). -1 invalid. */
typedef struct or_read_request {
  uint64_t group; /* global shard id */
  uint32_t slot, _pad;
  uint64_t ctx;   /* non-zero request context (dragonboat's SystemCtx) */
} or_read_request;
int or_read_index(or_engine* e, const or_read_request* reqs, size_t n);
/* The reads replica rid's last step made ready (ReadyToRead), in the order they became ready: returns
 * how many (at most OR_RQ), the first `cap` of them in ctx[] / index[] (serve each once applied >=
 * its index). */
int or_get_read_ready(const or_engine* e, uint32_t rid, uint64_t* ctx, uint64_t* index, uint32_t cap);
/* Snapshot events of rid's last step (the oracle side of rg_snapshot_events): OR_SNAP_* bits. */
#define OR_SNAP_TAKEN 1
#define OR_SNAP_RESTORED 2
/* Whole-table digest: out[0] = Σ over replicas of an fmix64 chain over the replica's
 * view (the or_replica_view fields, remotes of slots < R), out[1] = Σ of a chain over its log entries
 * (marker, last] (term, then type | len << 8 | crc << 32); each chain seeded by the global replica id.
 * Order-independent: the sum over ranks / windows is the digest of their union. Same function as
 * rg_digest. */
int or_digest(const or_engine* e, uint64_t out[2]);
int or_get_snapshot_event(const or_engine* e, uint32_t rid, uint64_t* restored, uint64_t* index, uint64_t* term);
/* the first index rid's last step handed to the state machine (tests: the engine's hand-off word) */
int or_debug_apply_lo(const or_engine* e, uint32_t rid, uint64_t* apply_lo);
/* Proposal payload generator: the synthetic Cmd of a tick-input proposal, len payload_bytes. */
void or_payload(const or_engine* e, uint32_t slab, uint32_t group, uint32_t entry, uint8_t* out);
uint32_t or_crc32(const uint8_t* p, size_t n);
uint32_t or_crc32c(const uint8_t* p, size_t n);
uint64_t or_mix64(uint64_t z);

#ifdef __cplusplus
}
#endif
#endif
