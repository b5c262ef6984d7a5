/*
 * abi_c.c — TEST HARNESS: drives libraftgpu.so through include/raftgpu.h from plain C, in the
 * call sequence the cgo NodeHost shim of INTEGRATION.md makes, with C-owned buffers only (cgo
 * forbids C from keeping Go pointers, so the shim copies into buffers like these):
 *
 *   rg_create / rg_bootstrap            NewNodeHost + StartOnDiskReplica (raft/raft_manager.go:109,142)
 *   rg_tick (campaign, then plain)      the NodeHost tick loop
 *   rg_propose                          NodeHost.SyncPropose(cmd) (the /raft/update handler's job)
 *   rg_get_update                       Peer.GetUpdate: in one hand-off the entries + State to persist
 *                                       (LogDB SaveRaftState before the messages leave) and the
 *                                       committed entries for IOnDiskStateMachine.Update → POST
 *                                       /UpdateEntries (INTEGRATION.md's per-tick call sequence)
 *   rg_commit_update(RG_COMMIT_APPLIED) Peer.Commit + NotifyRaftLastApplied once the app answered
 *   rg_apply_committed / rg_notify_applied  the same through the separate calls (drain phase)
 *   rg_config_change                    SyncRequestDeleteReplica / SyncRequestAddReplica (:165-185)
 *   rg_leader / rg_read_replicas        GetLeaderID / SyncGetShardMembership (raft/members.go:21,30)
 *   rg_destroy                          NodeHost.Close (raft_manager.go:159)
 *   rg_wire_exchange + rg_rccl_*        (argument "rccl") every message through the wire and the
 *                                       library's RCCL transport at world size 1: the multi-GPU
 *                                       replication path of a non-Python host
 *
 * Checks: every proposed Cmd reaches Update exactly once per replica, in proposal order, byte for
 * byte, with its zlib CRC-32 — including a follower removed from the membership for six ticks and
 * added back, which catches up; every shard has one leader and full membership at the end; errors
 * come back as RG_E* codes.
 * Exit 0 and "ABI_C OK" on success. Built by tests/test_abi.py (gcc, -lraftgpu -lz); run by the
 * -m gpu test there.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "../../include/raftgpu.h"

#define G 16
#define R 3
#define TICKS 40
#define PER_TICK 4 /* Cmds per shard per tick */
#define MAXC 1500  /* a usual Cmd: up to six 256-B lane groups, up to two pages */
#define LONGC 70000 /* about one Cmd in eleven: 8,192 .. LONGC bytes (past r03's 8,191-B ceiling) */

#define CHECK(x)                                                                              \
  do {                                                                                        \
    int _rc = (x);                                                                            \
    if (_rc < 0) {                                                                            \
      fprintf(stderr, "%s:%d: %s = %d (%s)\n", __FILE__, __LINE__, #x, _rc, rg_last_error()); \
      exit(1);                                                                                \
    }                                                                                         \
  } while (0)
#define EXPECT(c)                                                      \
  do {                                                                 \
    if (!(c)) {                                                        \
      fprintf(stderr, "%s:%d: expectation failed: %s\n", __FILE__, __LINE__, #c); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

/* The shim's copy of the Cmds it persisted (what it wrote to its WAL), per replica and log index, kept
 * until the entry is handed to Update: rg_get_update's committed section refers to them when it comes
 * with the persist section (include/raftgpu.h, RG_UPDATE_COMMITTED_CMDS). A ring of PCAP slots per
 * replica tagged with the index: a replica's unapplied window never exceeds its log capacity. */
#define PCAP 1024 /* = rg_config.log_capacity below */
typedef struct {
  uint64_t index;
  uint32_t len;
  uint8_t* data;
} pcmd_t;
static pcmd_t pstore[G * R][PCAP];
static void pstore_put(uint32_t rid, uint64_t index, const uint8_t* cmd, uint32_t len) {
  pcmd_t* p = &pstore[rid][index & (PCAP - 1)];
  free(p->data);
  p->index = index;
  p->len = len;
  p->data = (uint8_t*)malloc(len ? len : 1);
  memcpy(p->data, cmd, len);
}

/* The WAL writer's walk of a persistence batch (the shim fsyncs these): per replica its entries
 * first..last, their terms from the runs, each application Cmd at the replica's payload_off + the
 * rounded lengths before it; a ConfigChange's len is RG_PERSIST_CONFIG | its descriptor. Each Cmd is
 * also kept in pstore (above). */
static void persist_walk(const rg_persist_batch* b) {
  uint64_t seen = 0, tseen = 0;
  for (uint64_t s = 0; s < b->n_states; ++s) {
    const rg_persist_state* st = &b->states[s];
    const uint64_t n = st->first <= st->last ? st->last - st->first + 1 : 0;
    EXPECT(st->entry_off == seen && st->term_off == tseen);
    uint64_t cnt = 0, prev = 0;
    for (uint32_t k = 0; k < st->n_terms; ++k) {
      const rg_persist_term* t = &b->terms[st->term_off + k];
      EXPECT(t->count >= 1 && t->term > prev); /* terms only grow along a log */
      prev = t->term;
      cnt += t->count;
    }
    EXPECT(cnt == n);
    uint64_t off = st->payload_off;
    for (uint64_t k = 0; k < n; ++k) {
      const rg_persist_entry* p = &b->entries[st->entry_off + k];
      if (p->len & RG_PERSIST_CONFIG) continue;
      EXPECT(off + p->len <= b->payload_bytes);
      if (p->len) EXPECT(p->crc == (uint32_t)crc32(0, b->payload + off, p->len));
      pstore_put(st->rid, st->first + k, b->payload + off, p->len);
      off += (p->len + 15u) & ~15u;
    }
    seen += n;
    tseen += st->n_terms;
  }
  EXPECT(seen == b->n_entries && tseen == b->n_terms);
}

/* IOnDiskStateMachine.Update from a copy-back batch, the way a cgo shim walks it: per run, entry k is
 * index first + k, its Cmd at off + the 16-B-rounded lengths before it — or, when the batch came by
 * reference (payload NULL: rg_get_update with the persist section), the Cmd the shim persisted for that
 * replica and index; each replica's state machine receives its entries in index order (a running CRC
 * over the Cmds, the count, the longest Cmd) */
static void consume(const rg_apply_batch* b, uint64_t* got, uint32_t* got_crc, uint64_t* last_idx,
                    uint32_t* longest) {
  uint64_t seen = 0;
  for (uint64_t r = 0; r < b->n_runs; ++r) {
    const rg_apply_run* run = &b->runs[r];
    EXPECT(run->count >= 1 && run->entry == seen && run->entry + run->count <= b->n_entries);
    uint64_t off = run->off;
    for (uint32_t k = 0; k < run->count; ++k) {
      const rg_apply_cmd* c = &b->cmds[run->entry + k];
      const uint8_t* cmd;
      if (b->payload) {
        cmd = b->payload + off;
        EXPECT(off + c->len <= b->payload_bytes);
      } else {  /* by reference: the Cmd the shim persisted */
        const pcmd_t* p = &pstore[run->rid][(run->first + k) & (PCAP - 1)];
        EXPECT(b->payload_bytes == 0 && p->index == run->first + k && p->len == c->len);
        cmd = p->data;
      }
      EXPECT(c->crc == (uint32_t)crc32(0, cmd, c->len));
      EXPECT(run->first + k > last_idx[run->rid]);
      last_idx[run->rid] = run->first + k;
      got_crc[run->rid] = (uint32_t)crc32(got_crc[run->rid], cmd, c->len);
      got[run->rid]++;
      if (c->len > *longest) *longest = c->len;
      off += (c->len + 15u) & ~15u;
    }
    seen += run->count;
  }
  EXPECT(seen == b->n_entries);
}

/* deterministic Cmd k of shard g at tick t: "put g/t/k" + filler, 1..MAXC bytes (longer than
 * payload_bytes, so Cmds span lane groups and pages) */
static uint32_t make_cmd(uint32_t g, uint32_t t, uint32_t k, uint8_t* out) {
  uint32_t n = (uint32_t)snprintf((char*)out, 256, "put shard=%u tick=%u k=%u;", g, t, k);
  uint32_t len = 1 + (g * 131 + t * 31 + k * 7) % MAXC;
  if ((g + 3 * t + 5 * k) % 11 == 0) len = 8192 + (g * 977 + t * 131 + k * 17) % (LONGC - 8192);
  if (len < n) len = n;
  for (uint32_t i = n; i < len; ++i) out[i] = (uint8_t)('a' + (g + t + k + i) % 26);
  return len;
}

static rg_transport xt;
static int use_wire = 0;
static int ticks = 0;

/* the NodeHost tick: with the wire, the last tick's messages are exchanged first */
static int tick(rg_engine* e, const rg_tick_input* in) {
  if (use_wire && ticks > 0) {
    uint64_t sent = 0;
    int rc = rg_wire_exchange(e, &xt, &sent);
    if (rc < 0) return rc;
    if (sent != 0) return RG_EINVAL; /* one rank: its only region is its own */
  }
  ++ticks;
  return rg_tick(e, in);
}

int main(int argc, char** argv) {
  use_wire = argc > 1 && strcmp(argv[1], "rccl") == 0;
  rg_config c;
  memset(&c, 0, sizeof c);
  c.groups = G; c.replicas = R; c.log_capacity = 1024; c.payload_bytes = 256;
  c.max_cmd_bytes = 1u << 20;
  c.pool_pages = 16384; /* 64 MiB: the long Cmds of 40 ticks stay live (no compaction before 1,000 entries) */
  c.max_entries_per_msg = 16; c.max_msgs_per_pair = 8; c.num_slabs = 2;
  c.election_rtt = 10; c.heartbeat_rtt = 1; c.check_quorum = 1; /* raftd's config (raft_manager.go:92-100) */
  c.snapshot_entries = 1000; c.compaction_overhead = 5; c.seed = 0x5EED; c.ranks = 1;
  c.apply_feedback = 1;
  c.wire_all = (uint32_t)use_wire;
  if (use_wire) {
    uint8_t uid[128];
    CHECK(rg_rccl_unique_id(uid));
    CHECK(rg_rccl_open(uid, 1, 0, 0, &xt));
  }
  rg_engine* e = NULL;
  CHECK(rg_create(&c, &e));
  CHECK(rg_bootstrap(e));

  /* errors are codes, not crashes */
  rg_proposal bad = {G + 5, 0, 1, 0};
  uint32_t one = 1;
  EXPECT(rg_propose(e, &bad, 1, (const uint8_t*)"x", &one) == RG_EINVAL);
  EXPECT(rg_config_change(e, 0, 0, 7, 1) == RG_EINVAL);
  EXPECT(rg_last_error()[0] != 0);

  uint8_t campaign[G * R];
  memset(campaign, 0, sizeof campaign);
  rg_tick_input in;
  memset(&in, 0, sizeof in);
  CHECK(tick(e, &in));
  for (uint32_t g = 0; g < G; ++g) campaign[g * R + (g % R)] = 1;  /* leaders spread over the slots */
  in.campaign = campaign;
  /* every replica reports the bootstrap entries applied (the rsm applies config changes itself) */
  uint32_t rids[G * R];
  uint64_t idx[G * R];
  for (uint32_t r = 0; r < G * R; ++r) { rids[r] = r; idx[r] = R; }
  CHECK(rg_notify_applied(e, rids, idx, G * R));
  CHECK(tick(e, &in));
  in.campaign = NULL;
  for (int t = 0; t < 6; ++t) CHECK(tick(e, &in));

  /* what each replica's state machine received, as a running CRC over (index, Cmd) */
  uint64_t got[G * R];
  uint32_t got_crc[G * R];
  uint64_t last_idx[G * R];
  uint32_t longest = 0;
  memset(got, 0, sizeof got);
  memset(got_crc, 0, sizeof got_crc);
  memset(last_idx, 0, sizeof last_idx);

  uint8_t* blob = (uint8_t*)malloc(G * PER_TICK * LONGC);
  uint32_t lens[G * PER_TICK];
  rg_proposal props[G];
  uint32_t want_crc[G];
  uint64_t want_n[G];
  memset(want_crc, 0, sizeof want_crc);
  memset(want_n, 0, sizeof want_n);
  for (uint32_t t = 0; t < TICKS; ++t) {
    uint64_t off = 0;
    for (uint32_t g = 0; g < G; ++g) {
      uint64_t leader = 0, term = 0;
      int valid = 0;
      CHECK(rg_leader(e, g, &leader, &term, &valid));
      props[g].group = g;
      props[g].slot = valid ? (uint32_t)(leader - 1) : 0;
      props[g].count = PER_TICK;
      props[g].first = (uint64_t)g * PER_TICK;
      for (uint32_t k = 0; k < PER_TICK; ++k) {
        uint32_t n = make_cmd(g, t, k, blob + off);
        lens[g * PER_TICK + k] = n;
        off += n;
      }
    }
    CHECK(rg_propose(e, props, G, blob, lens));
    /* a follower leaves the membership and comes back six ticks later — within its election timeout
     * (no heartbeats reach a removed replica; one that timed out would campaign at a higher term and
     * depose the leader when re-added, as without PreVote in dragonboat) */
    if (t == 10 || t == 16)
      for (uint32_t g = 0; g < G; ++g)
        CHECK(rg_config_change(e, g, props[g].slot, t == 10 ? RG_CC_REMOVE : RG_CC_ADD, (props[g].slot + 2) % R));
    off = 0;
    for (uint32_t g = 0; g < G; ++g)
      for (uint32_t k = 0; k < PER_TICK; ++k) {
        uint32_t n = lens[g * PER_TICK + k];
        want_crc[g] = (uint32_t)crc32(want_crc[g], blob + off, n);
        want_n[g]++;
        off += n;
      }
    CHECK(tick(e, &in));
    /* Peer.GetUpdate: the whole hand-off of the tick in one call (engine-owned pinned sections) */
    rg_update u;
    CHECK(rg_get_update(e, 0xFF, RG_UPDATE_PERSIST | RG_UPDATE_COMMITTED, &u));
    EXPECT(u.tick == (uint64_t)ticks && u.persist.n_states > 0);
    EXPECT(u.committed.n_entries == 0 || (u.committed.payload == NULL && u.committed.payload_bytes == 0));
    persist_walk(&u.persist);
    consume(&u.committed, got, got_crc, last_idx, &longest);
    /* Peer.Commit: the app answered, applied = processed (config changes and no-ops included) */
    CHECK(rg_commit_update(e, &u, RG_COMMIT_APPLIED));
  }
  for (int t = 0; t < 16; ++t) { /* drain: the last Cmds commit everywhere, the re-added follower catches up */
    rg_apply_batch b;
    CHECK(tick(e, &in));
    CHECK(rg_apply_committed(e, 0xFF, &b));
    consume(&b, got, got_crc, last_idx, &longest);
    rg_replica_view v[G * R];
    CHECK(rg_read_replicas(e, 0, G * R, v));
    for (uint32_t r = 0; r < G * R; ++r) idx[r] = v[r].processed;
    CHECK(rg_notify_applied(e, rids, idx, G * R));
  }
  rg_replica_view v[G * R];
  CHECK(rg_read_replicas(e, 0, G * R, v));
  for (uint32_t g = 0; g < G; ++g) {
    uint32_t leaders = 0;
    for (uint32_t s = 0; s < R; ++s) {
      const uint32_t r = g * R + s;
      leaders += v[r].role == RG_LEADER;
      EXPECT(v[r].err == 0);
      EXPECT(v[r].members == (1u << R) - 1u);
      if (got[r] != want_n[g] || got_crc[r] != want_crc[g]) {
        fprintf(stderr, "shard %u replica %u: %llu Cmds crc %08x, want %llu crc %08x\n", g, s + 1,
                (unsigned long long)got[r], got_crc[r], (unsigned long long)want_n[g], want_crc[g]);
        return 1;
      }
    }
    EXPECT(leaders == 1);
  }
  EXPECT(longest > 8191); /* Cmds past the old 13-bit length field went through Update */
  uint64_t pages = 0, free_pages = 0;
  int pool_failed = 1;
  CHECK(rg_pool_stats(e, &pages, &free_pages, &pool_failed));
  EXPECT(!pool_failed && free_pages > 0);
  printf("ABI_C OK%s: %u shards x %u replicas, %llu Cmds per shard applied on every replica, device %.1f MB\n",
         use_wire ? " (wire + RCCL exchange)" : "", G, R, (unsigned long long)want_n[0], rg_device_bytes(e) / 1e6);
  rg_destroy(e);
  if (use_wire) CHECK(rg_rccl_close(&xt));
  free(blob);
  return 0;
}
