/*
 * oracle.c — CPU restatement of dragonboat v4 internal/raft per-shard step, as specified in
 * DESIGN.md §1 (= SURVEY.md Appendix A with its VERIFY points decided).
 *
 * TEST INFRASTRUCTURE ONLY (checker for the HIP engine, and bench.py's cpu_baseline leg).
 * PARITY UNPINNED against dragonboat (module github.com/lni/dragonboat/v4
 * v4.0.0-20240618143154-6a1623140f27 is absent; see oracle.h). Function names follow the
 * upstream functions they restate; each cites the SURVEY Appendix A section it follows.
 *
 * Structure: value semantics everywhere. Messages copy their entries (term, type, len, crc,
 * payload) into the sender's per-tick outbox arena; the receiver reads them in the next tick.
 * Groups are independent within a tick, so or_tick() runs groups on worker threads with
 * group g → worker g % T, the arrangement of dragonboat's step workers.
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

typedef struct {
  uint64_t term;
  uint32_t type, len, crc;
  uint32_t pos; /* payload stream position (16-B chunks) of its Cmd in the replica's log */
  uint64_t off; /* in an outbox or the proposal staging: byte offset of its Cmd in that arena */
} ent_t;

typedef struct {
  or_msg_view h;
  uint32_t ent_off; /* first entry in the sender's outbox arena */
} msg_t;

typedef struct {
  uint32_t n[OR_MAX_R];       /* enqueued messages per destination slot */
  uint32_t emitted[OR_MAX_R]; /* emissions per destination incl. lost ones (loss hash input) */
  msg_t* m;                   /* [R][K_MAX] */
  ent_t* ents;                /* entry arena for Replicate payload copies */
  uint8_t* pay;               /* their Cmds, back to back (ent_t.off) */
  size_t n_ents, cap_ents, pay_used, pay_cap;
} outbox_t;

typedef struct {
  uint64_t term, vote, leader, committed, applied, last, marker, marker_term;
  uint64_t snap_index, snap_term, cap_base;
  uint64_t processed; /* committed entries handed to the state machine (entryLog.processed) */
  uint32_t role, election_tick, heartbeat_tick, rand_timeout, rng_ctr;
  uint32_t granted, responded, active, err, drops;
  uint32_t members, snap_members, cc_pending; /* DESIGN §1.8 */
  uint64_t match[OR_MAX_R], next[OR_MAX_R], rsnap[OR_MAX_R];
  uint8_t rstate[OR_MAX_R];
  /* log ring: index i in (marker, last] lives at slot i & (L-1) */
  ent_t* log;
  uint8_t** cmd;    /* [L] the Cmd bytes of the entry at each ring slot (grown to its longest Cmd) */
  uint32_t* cmdcap; /* [L] */
  outbox_t ob[2];
  uint32_t g, s; /* group, slot */
  /* apply window of the last step: entries apply_lo .. processed went to the state machine
   * (rsm → IOnDiskStateMachine.Update); a range restored from a snapshot does not */
  uint64_t apply_lo, restored_at;
  int took; /* a snapshot was taken at the end of the last step */
  /* ReadIndex (dragonboat's readIndex: pending + queue): the leader's pending requests in arrival
   * order — ctx, the commit index when it arrived, the slots that confirmed it (itself included) and
   * the requester's slot — and the reads made ready in a step (rd_tick = step + 1) */
  uint32_t rq_n;
  uint64_t rq_ctx[OR_RQ], rq_index[OR_RQ];
  uint32_t rq_acks[OR_RQ], rq_from[OR_RQ];
  uint32_t rd_n;
  uint64_t rd_ctx[OR_RQ], rd_index[OR_RQ], rd_tick;
  /* payload stream: the capacity rule's state. hw = next free chunk; lpg = lowest page
   * held; fidx = the step compacted or restored below this entry: its position bounds the pages the
   * next step releases (nlpg, effective once that step ends) */
  uint32_t hw, lpg, nlpg;
  uint64_t fidx;
} rep_t;

struct or_engine {
  or_config c;
  uint32_t nrep;
  uint32_t maxc, pts; /* longest Cmd, stream pages per replica */
  rep_t* reps;
  uint64_t t; /* next tick to run */
  const or_tick_input* in;
  /* caller proposals staged for the next tick (or_propose), per window group */
  uint8_t* stg_slot;  /* [G] target slot, 0xFF none */
  uint32_t* stg_n;    /* [G] entries */
  ent_t* stg_ents;    /* [G][E] len and arena offset per entry */
  uint8_t* stg_pay;   /* the staged Cmds, back to back (ent_t.off) */
  size_t stg_used, stg_cap;
  int staged;
  uint64_t* rd_req;   /* [G*R] ReadIndex contexts staged for the next tick (0 none) */
  int rd_staged;
  uint8_t* cc_slot;   /* [G] membership change staged for the next tick: proposing slot (0xFF none) */
  uint8_t* cc_desc;   /* [G] its descriptor OR_CC(op, target) */
  int cc_staged;
};

/* ---------------------------------------------------------------- helpers */

uint64_t or_mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ULL;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return z;
}

uint32_t or_crc32(const uint8_t* p, size_t n) {
  /* zlib's crc32 = CRC-32/IEEE (reflected 0xEDB88320, init/xorout 0xFFFFFFFF) */
  return (uint32_t)crc32(0L, p, (uInt)n);
}

uint32_t or_crc32c(const uint8_t* p, size_t n) {
  /* CRC-32C (Castagnoli): reflected 0x82F63B78, init/xorout 0xFFFFFFFF, bit at a time (the
   * published definition; Go's hash/crc32 MakeTable(crc32.Castagnoli)) */
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
  }
  return c ^ 0xFFFFFFFFu;
}

static uint32_t entry_crc(const or_engine* e, const uint8_t* p, size_t n) {
  return e->c.crc32c ? or_crc32c(p, n) : or_crc32(p, n);
}

void or_payload(const or_engine* e, uint32_t slab, uint32_t group, uint32_t entry, uint8_t* out) {
  /* DESIGN §1.3 payload generator */
  uint64_t key = or_mix64(((uint64_t)slab << 56) ^ ((uint64_t)group << 16) ^ (uint64_t)entry ^
                          (e->c.seed * 0x9E3779B97F4A7C15ULL));
  uint32_t P = e->c.payload_bytes;
  for (uint32_t w = 0; w < P / 8; ++w) {
    uint64_t v = or_mix64(key + (uint64_t)(w + 1) * 0xD1B54A32D192ED03ULL);
    memcpy(out + 8 * w, &v, 8); /* little-endian host */
  }
}

static inline uint32_t id_of(uint32_t slot) { return slot + 1; }
static inline uint32_t slot_of(uint64_t id) { return (uint32_t)(id - 1); }
static inline uint32_t popc(uint32_t x) { return (uint32_t)__builtin_popcount(x); }
/* raft.quorum over the voting members (numVotingMembers / 2 + 1) */
static inline uint32_t quorum(const rep_t* r) { return popc(r->members) / 2 + 1; }
static inline int is_member(const rep_t* r, uint32_t slot) { return (r->members >> slot) & 1u; }
static inline uint64_t u64min(uint64_t a, uint64_t b) { return a < b ? a : b; }
static inline uint64_t u64max(uint64_t a, uint64_t b) { return a > b ? a : b; }
static inline ent_t* log_at(const or_engine* e, const rep_t* r, uint64_t i) {
  return &r->log[i & (e->c.log_capacity - 1)];
}
static inline const uint8_t* logpay_at(const or_engine* e, const rep_t* r, uint64_t i) {
  return r->cmd[i & (e->c.log_capacity - 1)];
}
/* the ring slot of index i, made to hold a Cmd of len bytes */
static uint8_t* logpay_put(const or_engine* e, rep_t* r, uint64_t i, uint32_t len) {
  const uint64_t k = i & (e->c.log_capacity - 1);
  if (r->cmdcap[k] < len) {
    r->cmd[k] = (uint8_t*)realloc(r->cmd[k], len);
    r->cmdcap[k] = len;
  }
  return r->cmd[k];
}
/* 16-B chunks a Cmd of len bytes takes in the payload stream */
static inline uint32_t chunks_of(uint32_t len) { return (len + 15u) >> 4; }
/* stream capacity rule: an append of c chunks fits iff its last chunk's page lies
 * within stream_pages of the lowest page still held (page numbers are positions >> 8, mod 2^24) */
static int stream_fits(const or_engine* e, const rep_t* r, uint32_t c) {
  if (c == 0) return 1;
  return ((((r->hw + c - 1u) >> 8) - r->lpg) & 0xFFFFFFu) < e->pts;
}

/* entryLog.term: (0, nil) outside [firstIndex-1, lastIndex]  (SURVEY A.9 / DESIGN §1.2) */
static uint64_t term_of(const or_engine* e, const rep_t* r, uint64_t i) {
  if (i == r->marker) return r->marker_term;
  if (i > r->marker && i <= r->last) return log_at(e, r, i)->term;
  return 0;
}
static int match_term(const or_engine* e, const rep_t* r, uint64_t i, uint64_t t) {
  return term_of(e, r, i) == t;
}
static uint64_t last_term(const or_engine* e, const rep_t* r) { return term_of(e, r, r->last); }
/* entryLog.upToDate (A.8) */
static int up_to_date(const or_engine* e, const rep_t* r, uint64_t i, uint64_t t) {
  uint64_t lt = last_term(e, r);
  return t > lt || (t == lt && i >= r->last);
}

static inline uint64_t global_group(const or_engine* e, const rep_t* r) { return (uint64_t)e->c.group_base + r->g; }

static uint32_t rand_timeout(const or_engine* e, const rep_t* r) {
  uint64_t key = (global_group(e, r) << 32) | ((uint64_t)r->s << 24) | (uint64_t)(r->rng_ctr & 0xFFFFFF);
  uint64_t v = or_mix64(e->c.seed ^ or_mix64(key));
  return e->c.election_rtt + (uint32_t)(v % e->c.election_rtt);
}

/* ---------------------------------------------------------------- outbox */

static int lost(const or_engine* e, const rep_t* r, uint32_t dst, uint32_t n) {
  const or_tick_input* in = e->in;
  uint32_t rid = r->g * e->c.replicas + r->s;
  if (in && in->isolate) {
    if (in->isolate[rid] || in->isolate[r->g * e->c.replicas + dst]) return 1;
  }
  if (e->c.drop_ppm) {
    uint64_t grid = global_group(e, r) * e->c.replicas + r->s;
    uint64_t h = or_mix64(e->c.seed ^ or_mix64((e->t << 40) ^ (grid << 8) ^ dst) ^ (uint64_t)(n + 1));
    if (h % 1000000ULL < e->c.drop_ppm) return 1;
  }
  return 0;
}

static outbox_t* cur_ob(const or_engine* e, rep_t* r) { return &r->ob[e->t & 1]; }

static void arena_reserve(const or_engine* e, outbox_t* ob, size_t need) {
  (void)e;
  if (ob->n_ents + need <= ob->cap_ents) return;
  size_t nc = ob->cap_ents ? ob->cap_ents * 2 : 256;
  while (nc < ob->n_ents + need) nc *= 2;
  ob->ents = (ent_t*)realloc(ob->ents, nc * sizeof(ent_t));
  ob->cap_ents = nc;
}

/* room for `bytes` more Cmd bytes in an arena; returns the offset they start at */
static uint64_t bytes_reserve(uint8_t** buf, size_t* used, size_t* cap, size_t bytes) {
  if (*used + bytes > *cap) {
    size_t nc = *cap ? *cap * 2 : 4096;
    while (nc < *used + bytes) nc *= 2;
    *buf = (uint8_t*)realloc(*buf, nc);
    *cap = nc;
  }
  uint64_t at = *used;
  *used += bytes;
  return at;
}

/* copy the Cmd of log index i (an entry view en) into the outbox arena: en->off */
static void ob_put_cmd(outbox_t* ob, ent_t* en, const uint8_t* src) {
  en->off = 0;
  if (!(en->type == OR_ENTRY_APP && en->len)) return;
  en->off = bytes_reserve(&ob->pay, &ob->pay_used, &ob->pay_cap, en->len);
  memcpy(ob->pay + en->off, src, en->len);
}

/* raft.send + transport enqueue. Returns the outbox slot or NULL if the message was lost. */
static msg_t* send_msg(or_engine* e, rep_t* r, or_msg_view* h) {
  uint32_t dst = slot_of(h->to);
  h->from = (uint8_t)id_of(r->s);
  if (h->type != OR_PROPOSE && h->type != OR_REQUEST_VOTE && h->type != OR_READ_INDEX) h->term = r->term;
  outbox_t* ob = cur_ob(e, r);
  uint32_t n = ob->emitted[dst]++;
  if (lost(e, r, dst, n) || ob->n[dst] >= e->c.max_msgs_per_pair) {
    r->drops++;
    return NULL;
  }
  msg_t* m = &ob->m[dst * e->c.max_msgs_per_pair + ob->n[dst]++];
  m->h = *h;
  m->ent_off = 0;
  return m;
}

/* ---------------------------------------------------------------- role transitions (A.5) */

static void reset(or_engine* e, rep_t* r, uint64_t t) {
  if (t != r->term) {
    r->term = t;
    r->vote = 0;
  }
  r->leader = 0;
  r->granted = r->responded = 0;
  r->election_tick = r->heartbeat_tick = 0;
  r->rng_ctr++;
  r->rand_timeout = rand_timeout(e, r);
  for (uint32_t i = 0; i < e->c.replicas; ++i) {
    r->match[i] = 0;
    r->next[i] = r->last + 1;
    r->rsnap[i] = 0;
    r->rstate[i] = OR_RETRY;
  }
  r->match[r->s] = r->last;
  r->active = 0;
  r->rq_n = 0;       /* readIndex.reset: a new readIndex */
  r->cc_pending = 0; /* clearPendingConfigChange */
}

static void become_follower(or_engine* e, rep_t* r, uint64_t t, uint64_t leader) {
  r->role = OR_FOLLOWER;
  reset(e, r, t);
  r->leader = leader;
}

static void become_candidate(or_engine* e, rep_t* r) {
  r->role = OR_CANDIDATE;
  reset(e, r, r->term + 1);
  r->leader = 0;
  r->vote = id_of(r->s);
}

static int try_commit(or_engine* e, rep_t* r);
static void broadcast_replicate(or_engine* e, rep_t* r);

/* remote.tryUpdate (A.10) */
static int remote_try_update(rep_t* r, uint32_t i, uint64_t idx) {
  if (r->next[i] < idx + 1) r->next[i] = idx + 1;
  if (r->match[i] < idx) {
    if (r->rstate[i] == OR_WAIT) r->rstate[i] = OR_RETRY;
    r->match[i] = idx;
    return 1;
  }
  return 0;
}

/* Where the Cmds of an append come from: the entries a Propose message
 * carries (ents / pay, entry k's Cmd at pay + ents[k].off), or, for a tick-input proposal, the synthetic generator
 * (slab >= 0: Cmd k = or_payload(slab, group, k), len P). NULL source: len-0 no-ops. cc != 0: one
 * ConfigChange entry with that descriptor. */
typedef struct {
  int slab;
  const ent_t* ents;
  const uint8_t* pay;
  uint32_t cc;
} src_t;

/* raft.appendEntries: n entries at term. Returns 0 when the batch was refused by the capacity rule. */
static int append_entries(or_engine* e, rep_t* r, uint32_t n, const src_t* src) {
  uint32_t L = e->c.log_capacity, P = e->c.payload_bytes;
  if (r->last + n > r->cap_base + L) return 0;
  uint32_t c = 0; /* the batch's stream chunks (the capacity rule's input) */
  if (src && !src->cc && P)
    for (uint32_t k = 0; k < n; ++k) c += chunks_of(src->ents ? src->ents[k].len : P);
  if (!stream_fits(e, r, c)) return 0;
  for (uint32_t k = 0; k < n; ++k) {
    uint64_t idx = r->last + 1 + k;
    ent_t* en = log_at(e, r, idx);
    en->term = r->term;
    en->type = OR_ENTRY_APP;
    en->pos = r->hw;
    if (src && src->cc) { /* a ConfigChange entry: no Cmd, its descriptor in len */
      en->type = OR_ENTRY_CONFIG;
      en->len = src->cc;
      en->crc = 0;
      continue;
    }
    uint32_t len = !src || !P ? 0 : src->ents ? src->ents[k].len : P;
    if (len) {
      uint8_t* dst = logpay_put(e, r, idx, len);
      if (src->ents) memcpy(dst, src->pay + src->ents[k].off, len);
      else or_payload(e, (uint32_t)src->slab, (uint32_t)global_group(e, r), k, dst);
      en->len = len;
      en->crc = entry_crc(e, dst, len);
      r->hw += chunks_of(len);
    } else {
      en->len = 0;
      en->crc = 0;
    }
  }
  r->last += n;
  remote_try_update(r, r->s, r->last);
  if (popc(r->members) == 1) try_commit(e, r); /* isSingleNodeQuorum */
  return 1;
}

static void become_leader(or_engine* e, rep_t* r) {
  r->role = OR_LEADER;
  reset(e, r, r->term);
  r->leader = id_of(r->s);
  /* preLeaderPromotionHandleConfigChange: a ConfigChange entry in (committed, last] is in flight */
  for (uint64_t i = r->committed + 1; i <= r->last; ++i)
    if (log_at(e, r, i)->type == OR_ENTRY_CONFIG) r->cc_pending = 1;
  if (!append_entries(e, r, 1, NULL)) r->err |= OR_ERR_RING_FULL;
}

/* ---------------------------------------------------------------- leader replication (A.12) */

static void remote_progress(rep_t* r, uint32_t i, uint64_t last_sent) {
  if (r->rstate[i] == OR_REPLICATE_ST) r->next[i] = last_sent + 1;
  else if (r->rstate[i] == OR_RETRY) r->rstate[i] = OR_WAIT;
}

static void send_replicate(or_engine* e, rep_t* r, uint32_t to) {
  if (r->rstate[to] == OR_WAIT || r->rstate[to] == OR_SNAPSHOT) return;
  uint64_t next = r->next[to];
  or_msg_view h;
  memset(&h, 0, sizeof h);
  h.to = (uint8_t)id_of(to);
  if (next <= r->marker) { /* log compacted below next: InstallSnapshot path */
    if (!(r->active & (1u << to))) return;
    if (r->snap_index == 0) {
      r->err |= OR_ERR_EMPTY_SNAPSHOT;
      return;
    }
    h.type = OR_INSTALL_SNAPSHOT;
    h.log_index = r->snap_index;
    h.log_term = r->snap_term;
    h.hint_high = r->snap_members; /* the snapshot's membership */
    r->rsnap[to] = r->snap_index;
    r->rstate[to] = OR_SNAPSHOT;
    send_msg(e, r, &h);
    return;
  }
  uint32_t n = 0;
  if (next <= r->last) n = (uint32_t)u64min(e->c.max_entries_per_msg, r->last - next + 1);
  h.type = OR_REPLICATE;
  h.log_index = next - 1;
  h.log_term = term_of(e, r, next - 1);
  h.commit = r->committed;
  h.nent = n;
  if (n > 0) remote_progress(r, to, next + n - 1);
  msg_t* m = send_msg(e, r, &h);
  if (m && n) {
    outbox_t* ob = cur_ob(e, r);
    arena_reserve(e, ob, n);
    m->ent_off = (uint32_t)ob->n_ents;
    for (uint32_t k = 0; k < n; ++k) {
      ent_t* en = &ob->ents[ob->n_ents + k];
      *en = *log_at(e, r, next + k);
      if (e->c.payload_bytes) ob_put_cmd(ob, en, logpay_at(e, r, next + k));
    }
    ob->n_ents += n;
  }
}

static void broadcast_replicate(or_engine* e, rep_t* r) {
  for (uint32_t i = 0; i < e->c.replicas; ++i)
    if (i != r->s && is_member(r, i)) send_replicate(e, r, i);
}

static void broadcast_heartbeat(or_engine* e, rep_t* r) {
  for (uint32_t i = 0; i < e->c.replicas; ++i) {
    if (i == r->s || !is_member(r, i)) continue;
    or_msg_view h;
    memset(&h, 0, sizeof h);
    h.type = OR_HEARTBEAT;
    h.to = (uint8_t)id_of(i);
    h.commit = u64min(r->match[i], r->committed);
    h.hint = r->rq_n ? r->rq_ctx[r->rq_n - 1] : 0; /* readIndex.peepCtx: the newest pending request */
    send_msg(e, r, &h);
  }
}

/* raft.tryCommit + sortMatchValues + entryLog.tryCommit (A.13) */
static int try_commit(or_engine* e, rep_t* r) {
  uint32_t R = 0; /* the voting members' match values */
  uint64_t v[OR_MAX_R];
  for (uint32_t i = 0; i < e->c.replicas; ++i)
    if (is_member(r, i)) v[R++] = r->match[i];
  if (R == 0) return 0;
  for (uint32_t i = 1; i < R; ++i) { /* insertion sort ascending */
    uint64_t x = v[i];
    int j = (int)i - 1;
    while (j >= 0 && v[j] > x) {
      v[j + 1] = v[j];
      --j;
    }
    v[j + 1] = x;
  }
  uint64_t q = v[R - quorum(r)];
  if (q > r->committed && term_of(e, r, q) == r->term) {
    r->committed = q;
    return 1;
  }
  return 0;
}

/* ---------------------------------------------------------------- follower side (A.9) */

static void commit_to(rep_t* r, uint64_t i) {
  if (i <= r->committed) return;
  if (i > r->last) {
    r->err |= OR_ERR_COMMIT_BEYOND_LAST;
    return;
  }
  r->committed = i;
}

typedef struct {
  or_msg_view h;
  const ent_t* ents; /* Replicate / Propose entries (NULL: a tick-input proposal, synthetic Cmds) */
  const uint8_t* pay;
} msg_in_t;

static void handle_replicate(or_engine* e, rep_t* r, const msg_in_t* m) {
  uint32_t L = e->c.log_capacity, P = e->c.payload_bytes;
  or_msg_view resp;
  memset(&resp, 0, sizeof resp);
  resp.type = OR_REPLICATE_RESP;
  resp.to = m->h.from;
  if (m->h.log_index < r->committed) {
    resp.log_index = r->committed;
    send_msg(e, r, &resp);
    return;
  }
  uint32_t n = m->h.nent;
  if (match_term(e, r, m->h.log_index, m->h.log_term)) {
    /* entryLog.getConflictIndex */
    uint64_t ci = 0;
    uint32_t k0 = 0;
    for (uint32_t k = 0; k < n; ++k) {
      uint64_t idx = m->h.log_index + 1 + k;
      if (!match_term(e, r, idx, m->ents[k].term)) {
        ci = idx;
        k0 = k;
        break;
      }
    }
    uint64_t last_new = m->h.log_index + n;
    if (ci != 0 && ci > r->committed) { /* capacity rules (ring, then payload stream): dropped, no reply */
      uint32_t c = 0;
      for (uint32_t k = k0; k < n && P; ++k)
        if (m->ents[k].type == OR_ENTRY_APP) c += chunks_of(m->ents[k].len);
      if (last_new > r->cap_base + L || !stream_fits(e, r, c)) {
        r->drops++;
        return;
      }
    }
    if (ci != 0) {
      if (ci <= r->committed) {
        r->err |= OR_ERR_CONFLICT_COMMITTED;
      } else { /* entryLog.tryAppend → inMemory.merge: truncate at ci, append */
        for (uint32_t k = k0; k < n; ++k) {
          uint64_t idx = m->h.log_index + 1 + k;
          ent_t* en = log_at(e, r, idx);
          const ent_t* src = &m->ents[k];
          en->term = src->term;
          en->type = src->type;
          en->len = src->len;
          en->pos = r->hw;
          if (src->len && src->type == OR_ENTRY_APP) {
            uint8_t* dst = logpay_put(e, r, idx, src->len);
            memcpy(dst, m->pay + src->off, src->len);
            en->crc = entry_crc(e, dst, src->len);
            if (en->crc != src->crc) r->err |= OR_ERR_CRC;
            r->hw += chunks_of(src->len);
          } else {
            en->crc = 0;
          }
        }
        r->last = last_new;
      }
    }
    commit_to(r, u64min(last_new, m->h.commit));
    resp.log_index = last_new;
  } else {
    resp.reject = 1;
    resp.log_index = m->h.log_index;
    resp.hint = r->last;
  }
  send_msg(e, r, &resp);
}

static void handle_heartbeat(or_engine* e, rep_t* r, const or_msg_view* m) {
  commit_to(r, m->commit);
  or_msg_view resp;
  memset(&resp, 0, sizeof resp);
  resp.type = OR_HEARTBEAT_RESP;
  resp.to = m->from;
  resp.hint = m->hint;
  resp.hint_high = m->hint_high;
  send_msg(e, r, &resp);
}

static void handle_install_snapshot(or_engine* e, rep_t* r, const or_msg_view* m) {
  or_msg_view resp;
  memset(&resp, 0, sizeof resp);
  resp.type = OR_REPLICATE_RESP;
  resp.to = m->from;
  uint64_t si = m->log_index, st = m->log_term;
  if (si <= r->committed) {
    resp.log_index = r->committed;
  } else if (match_term(e, r, si, st)) {
    commit_to(r, si);
    resp.log_index = r->committed;
  } else { /* raft.restore → entryLog.restore; the state machine recovers from the snapshot */
    r->marker = r->last = r->committed = r->snap_index = r->processed = si;
    r->marker_term = r->snap_term = st;
    r->applied = u64max(r->applied, si);
    r->members = r->snap_members = (uint32_t)m->hint_high; /* the snapshot's membership */
    resp.log_index = r->last;
    r->restored_at = si;
  }
  send_msg(e, r, &resp);
}

/* ---------------------------------------------------------------- elections (A.7, A.8) */

static void handle_vote_resp(rep_t* r, uint32_t from_slot, int rejected) {
  uint32_t bit = 1u << from_slot;
  if (!(r->responded & bit)) {
    r->responded |= bit;
    if (!rejected) r->granted |= bit;
  }
}

static void campaign(or_engine* e, rep_t* r) {
  become_candidate(e, r);
  handle_vote_resp(r, r->s, 0);
  if (popc(r->granted & r->members) == quorum(r)) { /* single-node quorum */
    become_leader(e, r);
    return;
  }
  for (uint32_t i = 0; i < e->c.replicas; ++i) {
    if (i == r->s || !is_member(r, i)) continue;
    or_msg_view h;
    memset(&h, 0, sizeof h);
    h.type = OR_REQUEST_VOTE;
    h.to = (uint8_t)id_of(i);
    h.term = r->term;
    h.log_index = r->last;
    h.log_term = last_term(e, r);
    send_msg(e, r, &h);
  }
}

static void handle_node_election(or_engine* e, rep_t* r) {
  if (r->role == OR_LEADER) return;
  if (!is_member(r, r->s)) return; /* selfRemoved: no elections */
  if (r->committed > r->applied) return; /* hasConfigChangeToApply */
  if (r->term >= OR_TERM_MAX) { /* the next term would not fit the ring word's 36-bit field */
    r->err |= OR_ERR_TERM_LIMIT;
    return;
  }
  campaign(e, r);
}

static void handle_node_request_vote(or_engine* e, rep_t* r, const or_msg_view* m) {
  or_msg_view resp;
  memset(&resp, 0, sizeof resp);
  resp.type = OR_REQUEST_VOTE_RESP;
  resp.to = m->from;
  int can_grant = r->vote == 0 || r->vote == m->from;
  if (can_grant && up_to_date(e, r, m->log_index, m->log_term)) {
    r->election_tick = 0;
    r->vote = m->from;
  } else {
    resp.reject = 1;
  }
  send_msg(e, r, &resp);
}

static void handle_candidate_vote_resp(or_engine* e, rep_t* r, const or_msg_view* m) {
  handle_vote_resp(r, slot_of(m->from), m->reject);
  uint32_t granted = popc(r->granted & r->members), total = popc(r->responded & r->members);
  if (granted == quorum(r)) {
    become_leader(e, r);
    broadcast_replicate(e, r);
  } else if (total - granted == quorum(r)) {
    become_follower(e, r, r->term, 0);
  }
}

/* ---------------------------------------------------------------- leader responses (A.10, A.11) */

static void handle_leader_replicate_resp(or_engine* e, rep_t* r, const or_msg_view* m) {
  uint32_t f = slot_of(m->from);
  if (!is_member(r, f)) return; /* no remote for it */
  r->active |= 1u << f;
  if (!m->reject) {
    int paused = r->rstate[f] == OR_WAIT || r->rstate[f] == OR_SNAPSHOT;
    if (remote_try_update(r, f, m->log_index)) {
      /* remote.respondedTo */
      if (r->rstate[f] == OR_RETRY) {
        r->next[f] = r->match[f] + 1;
        r->rsnap[f] = 0;
        r->rstate[f] = OR_REPLICATE_ST;
      } else if (r->rstate[f] == OR_SNAPSHOT && r->match[f] >= r->rsnap[f]) {
        r->next[f] = u64max(r->match[f] + 1, r->rsnap[f] + 1);
        r->rsnap[f] = 0;
        r->rstate[f] = OR_RETRY;
      }
      if (try_commit(e, r)) broadcast_replicate(e, r);
      else if (paused) send_replicate(e, r, f);
    }
  } else {
    /* remote.decreaseTo */
    uint64_t rej = m->log_index, hint = m->hint;
    int ok;
    if (r->rstate[f] == OR_REPLICATE_ST) {
      if (rej <= r->match[f]) ok = 0;
      else {
        r->next[f] = r->match[f] + 1;
        ok = 1;
      }
    } else if (r->next[f] - 1 != rej) {
      ok = 0;
    } else {
      if (r->rstate[f] == OR_WAIT) r->rstate[f] = OR_RETRY;
      r->next[f] = u64max(1, u64min(rej, hint + 1));
      ok = 1;
    }
    if (ok) {
      if (r->rstate[f] == OR_REPLICATE_ST) { /* enterRetryState → becomeRetry */
        r->next[f] = r->match[f] + 1;
        r->rsnap[f] = 0;
        r->rstate[f] = OR_RETRY;
      }
      send_replicate(e, r, f);
    }
  }
}

static void read_ready(or_engine* e, rep_t* r, uint64_t ctx, uint64_t index) { /* addReadyToRead */
  if (r->rd_tick != e->t + 1) {  /* the first read made ready in this step */
    r->rd_tick = e->t + 1;
    r->rd_n = 0;
  }
  if (r->rd_n == OR_RQ) { /* the step's ready list is full: dropped (counted) */
    r->drops++;
    return;
  }
  r->rd_ctx[r->rd_n] = ctx;
  r->rd_index[r->rd_n] = index;
  r->rd_n++;
}

/* the leader's confirmed read goes to its requester: itself, or a follower (ReadIndexResp) */
static void read_confirmed(or_engine* e, rep_t* r, uint64_t ctx, uint64_t index, uint32_t from_slot) {
  if (from_slot == r->s) {
    read_ready(e, r, ctx, index);
  } else {
    or_msg_view h;
    memset(&h, 0, sizeof h);
    h.type = OR_READ_INDEX_RESP;
    h.to = (uint8_t)id_of(from_slot);
    h.log_index = index;
    h.hint = ctx;
    send_msg(e, r, &h);
  }
}

static void handle_leader_heartbeat_resp(or_engine* e, rep_t* r, const or_msg_view* m) {
  uint32_t f = slot_of(m->from);
  if (!is_member(r, f)) return; /* no remote for it */
  r->active |= 1u << f;
  if (r->rstate[f] == OR_WAIT) r->rstate[f] = OR_RETRY;
  if (r->match[f] < r->last) send_replicate(e, r, f);
  if (m->hint == 0) return;
  /* readIndex.confirm: the request this heartbeat answered; once a quorum confirmed it, it and every
   * request queued before it are done, all at its index (dragonboat rewrites v.index = s.index) */
  uint32_t k = 0;
  while (k < r->rq_n && r->rq_ctx[k] != m->hint) ++k;
  if (k == r->rq_n) return;
  r->rq_acks[k] |= 1u << f;
  if (popc(r->rq_acks[k] & r->members) < quorum(r)) return;
  const uint64_t index = r->rq_index[k];
  uint64_t ctx[OR_RQ];
  uint32_t from[OR_RQ];
  for (uint32_t i = 0; i <= k; ++i) {
    ctx[i] = r->rq_ctx[i];
    from[i] = r->rq_from[i];
  }
  for (uint32_t i = k + 1; i < r->rq_n; ++i) { /* the rest move to the front */
    r->rq_ctx[i - k - 1] = r->rq_ctx[i];
    r->rq_index[i - k - 1] = r->rq_index[i];
    r->rq_acks[i - k - 1] = r->rq_acks[i];
    r->rq_from[i - k - 1] = r->rq_from[i];
  }
  r->rq_n -= k + 1;
  for (uint32_t i = 0; i <= k; ++i) read_confirmed(e, r, ctx[i], index, from[i]);
}

/* ReadIndex{hint = ctx} from slot m->from (itself, or a follower that forwarded it) */
static void handle_read_index(or_engine* e, rep_t* r, const or_msg_view* m) {
  uint32_t f = slot_of(m->from);
  if (r->role == OR_LEADER) {
    if (quorum(r) == 1) { /* isSingleNodeQuorum */
      read_confirmed(e, r, m->hint, r->committed, f);
    } else if (term_of(e, r, r->committed) != r->term) {
      r->drops++; /* no entry committed in this term yet (thesis §6.4) */
    } else {
      uint32_t k = 0; /* readIndex.addRequest: a context already pending is not added again */
      while (k < r->rq_n && r->rq_ctx[k] != m->hint) ++k;
      if (k == r->rq_n) {
        if (r->rq_n == OR_RQ) { /* the queue is full: dropped (counted), no heartbeat */
          r->drops++;
          return;
        }
        r->rq_ctx[k] = m->hint;
        r->rq_index[k] = r->committed;
        r->rq_acks[k] = 1u << r->s;
        r->rq_from[k] = f;
        r->rq_n++;
      }
      for (uint32_t i = 0; i < e->c.replicas; ++i) { /* broadcastHeartbeatMessageWithHint */
        if (i == r->s || !is_member(r, i)) continue;
        or_msg_view h;
        memset(&h, 0, sizeof h);
        h.type = OR_HEARTBEAT;
        h.to = (uint8_t)id_of(i);
        h.commit = u64min(r->match[i], r->committed);
        h.hint = m->hint;
        send_msg(e, r, &h);
      }
    }
  } else if (r->role == OR_FOLLOWER && r->leader != 0 && f == r->s) {
    or_msg_view h = *m;
    h.to = (uint8_t)r->leader;
    h.term = 0;
    send_msg(e, r, &h);
  } else {
    r->drops++;
  }
}

static void handle_leader_check_quorum(or_engine* e, rep_t* r) {
  uint32_t c = popc((r->active | (1u << r->s)) & r->members); /* leaderHasQuorum */
  r->active = 0;
  if (c < quorum(r)) become_follower(e, r, r->term, 0);
}

/* ---------------------------------------------------------------- proposals */

/* leader: appendEntries + broadcast; follower with a known leader: forward the proposal with its
 * entries (hop limit 1); otherwise dropped */
static void handle_propose(or_engine* e, rep_t* r, const msg_in_t* mi) {
  const or_msg_view* m = &mi->h;
  uint32_t P = e->c.payload_bytes;
  const uint32_t cc = (uint32_t)m->hint_high; /* a membership change: one entry */
  src_t src = {(int)m->src_a, mi->ents, mi->pay, cc};
  if (r->role == OR_LEADER) {
    int dropped_cc = 0;
    if (cc && r->cc_pending) { /* one change at a time: it becomes an empty application entry */
      src.cc = 0;
      src.ents = NULL;
      src.slab = -1;
      dropped_cc = 1;
    }
    if (!append_entries(e, r, m->nent, dropped_cc ? NULL : &src)) {
      r->drops++;
      return;
    }
    if (dropped_cc) r->drops++;          /* reportDroppedConfigChange */
    else if (cc) r->cc_pending = 1;      /* setPendingConfigChange */
    broadcast_replicate(e, r);
  } else if (r->role == OR_FOLLOWER && r->leader != 0 && m->src_b == 0) {
    or_msg_view h = *m;
    h.to = (uint8_t)r->leader;
    h.term = 0;
    h.src_b = m->src_b + 1;
    msg_t* fm = send_msg(e, r, &h);
    if (fm && P && m->nent && !cc) { /* the message carries its Cmds */
      outbox_t* ob = cur_ob(e, r);
      arena_reserve(e, ob, m->nent);
      fm->ent_off = (uint32_t)ob->n_ents;
      for (uint32_t k = 0; k < m->nent; ++k) {
        ent_t* en = &ob->ents[ob->n_ents + k];
        memset(en, 0, sizeof *en);
        en->type = OR_ENTRY_APP;
        en->len = mi->ents ? mi->ents[k].len : P;
        if (!en->len) continue;
        en->off = bytes_reserve(&ob->pay, &ob->pay_used, &ob->pay_cap, en->len);
        if (mi->ents) memcpy(ob->pay + en->off, mi->pay + mi->ents[k].off, en->len);
        else or_payload(e, m->src_a, (uint32_t)global_group(e, r), k, ob->pay + en->off);
      }
      ob->n_ents += m->nent;
    }
  } else {
    r->drops++;
  }
}

/* ---------------------------------------------------------------- Handle (A.3) */

static void handle(or_engine* e, rep_t* r, const msg_in_t* mi);

static void local(or_engine* e, rep_t* r, uint32_t type) {
  msg_in_t mi;
  memset(&mi, 0, sizeof mi);
  mi.h.type = (uint8_t)type;
  mi.h.from = (uint8_t)id_of(r->s);
  handle(e, r, &mi);
}

static void tick(or_engine* e, rep_t* r) {
  if (r->role == OR_LEADER) { /* leaderTick */
    r->election_tick++;
    if (r->election_tick >= e->c.election_rtt) {
      r->election_tick = 0;
      if (e->c.check_quorum) local(e, r, OR_CHECK_QUORUM);
    }
    r->heartbeat_tick++;
    if (r->heartbeat_tick >= e->c.heartbeat_rtt) {
      r->heartbeat_tick = 0;
      local(e, r, OR_LEADER_HEARTBEAT);
    }
  } else { /* nonLeaderTick: a replica outside the membership never starts an election */
    r->election_tick++;
    if (is_member(r, r->s) && r->election_tick >= r->rand_timeout) {
      r->election_tick = 0;
      local(e, r, OR_ELECTION);
    }
  }
}

static int is_leader_msg(uint32_t t) {
  return t == OR_REPLICATE || t == OR_INSTALL_SNAPSHOT || t == OR_HEARTBEAT || t == OR_READ_INDEX_RESP;
}

static void handle(or_engine* e, rep_t* r, const msg_in_t* mi) {
  const or_msg_view* m = &mi->h;
  if (m->term != 0 && m->term != r->term) {
    if (m->type == OR_REQUEST_VOTE && e->c.check_quorum && m->term > r->term && m->hint != m->from &&
        r->leader != 0 && r->election_tick < e->c.election_rtt)
      return; /* dropRequestVoteFromHighTermNode */
    if (m->term > r->term) {
      become_follower(e, r, m->term, is_leader_msg(m->type) ? m->from : 0);
    } else {
      if (e->c.check_quorum && is_leader_msg(m->type)) {
        or_msg_view h;
        memset(&h, 0, sizeof h);
        h.type = OR_NOOP;
        h.to = m->from;
        send_msg(e, r, &h);
      }
      return;
    }
  }
  switch (m->type) {
    case OR_LOCAL_TICK: tick(e, r); break;
    case OR_ELECTION: handle_node_election(e, r); break;
    case OR_LEADER_HEARTBEAT:
      if (r->role == OR_LEADER) broadcast_heartbeat(e, r);
      break;
    case OR_CHECK_QUORUM:
      if (r->role == OR_LEADER) handle_leader_check_quorum(e, r);
      break;
    case OR_PROPOSE: handle_propose(e, r, mi); break;
    case OR_REPLICATE:
      if (r->role == OR_LEADER) break;
      if (r->role == OR_CANDIDATE) become_follower(e, r, r->term, m->from);
      else {
        r->election_tick = 0;
        r->leader = m->from;
      }
      handle_replicate(e, r, mi);
      break;
    case OR_HEARTBEAT:
      if (r->role == OR_LEADER) break;
      if (r->role == OR_CANDIDATE) become_follower(e, r, r->term, m->from);
      else {
        r->election_tick = 0;
        r->leader = m->from;
      }
      handle_heartbeat(e, r, m);
      break;
    case OR_INSTALL_SNAPSHOT:
      if (r->role == OR_LEADER) break;
      if (r->role == OR_CANDIDATE) become_follower(e, r, r->term, m->from);
      else {
        r->election_tick = 0;
        r->leader = m->from;
      }
      handle_install_snapshot(e, r, m);
      break;
    case OR_REPLICATE_RESP:
      if (r->role == OR_LEADER) handle_leader_replicate_resp(e, r, m);
      break;
    case OR_HEARTBEAT_RESP:
      if (r->role == OR_LEADER) handle_leader_heartbeat_resp(e, r, m);
      break;
    case OR_READ_INDEX: handle_read_index(e, r, m); break;
    case OR_READ_INDEX_RESP:
      if (r->role == OR_FOLLOWER) {
        r->election_tick = 0; /* a leader message: like Heartbeat */
        r->leader = m->from;
        read_ready(e, r, m->hint, m->log_index);
      }
      break;
    case OR_REQUEST_VOTE: handle_node_request_vote(e, r, m); break;
    case OR_REQUEST_VOTE_RESP:
      if (r->role == OR_CANDIDATE) handle_candidate_vote_resp(e, r, m);
      break;
    default: break;
  }
}

/* ---------------------------------------------------------------- membership */

/* raft.addNode / raft.removeNode, reached through the rsm's ApplyConfigChange */
static void apply_config_change(or_engine* e, rep_t* r, uint32_t cc) {
  uint32_t op = cc >> 4, slot = (cc & 0xFu) - 1u;
  r->cc_pending = 0; /* clearPendingConfigChange */
  if (slot >= e->c.replicas) return;
  uint32_t bit = 1u << slot;
  if (op == OR_CC_ADD) {
    if (r->members & bit) return;
    r->members |= bit; /* setRemote(id, 0, lastIndex + 1) */
    r->match[slot] = 0;
    r->next[slot] = r->last + 1;
    r->rsnap[slot] = 0;
    r->rstate[slot] = OR_RETRY;
  } else if (op == OR_CC_REMOVE) {
    r->members &= ~bit; /* deleteRemote */
    r->active &= ~bit;
    if (slot == r->s && r->role == OR_LEADER) become_follower(e, r, r->term, 0);
    if (r->role == OR_LEADER && r->members && try_commit(e, r)) broadcast_replicate(e, r);
  }
}

/* ---------------------------------------------------------------- tick driver */

static void step_replica(or_engine* e, rep_t* r) {
  const or_tick_input* in = e->in;
  uint32_t R = e->c.replicas, K = e->c.max_msgs_per_pair;
  uint64_t marker_start = r->marker, processed_start = r->processed;
  r->restored_at = 0;
  r->took = 0;
  /* the pages below the last step's compaction / restore are released when this step ends */
  r->nlpg = r->lpg;
  if (r->fidx) r->nlpg = (r->fidx <= r->last ? log_at(e, r, r->fidx)->pos : r->hw) >> 8;
  outbox_t* ob = cur_ob(e, r);
  memset(ob->n, 0, sizeof ob->n);
  memset(ob->emitted, 0, sizeof ob->emitted);
  ob->n_ents = 0;
  ob->pay_used = 0;
  rep_t* grp = &e->reps[r->g * R];
  /* 1. inbound messages: source slot ascending, emission order */
  for (uint32_t src = 0; src < R; ++src) {
    if (src == r->s) continue;
    const outbox_t* sob = &grp[src].ob[(e->t + 1) & 1];
    for (uint32_t k = 0; k < sob->n[r->s]; ++k) {
      const msg_t* m = &sob->m[r->s * K + k];
      msg_in_t mi;
      mi.h = m->h;
      mi.ents = sob->ents + m->ent_off;
      mi.pay = sob->pay;
      handle(e, r, &mi);
    }
  }
  uint32_t rid = r->g * R + r->s;
  /* 2. campaign input */
  if (in && in->campaign && in->campaign[rid]) local(e, r, OR_ELECTION);
  /* 3. LocalTick */
  if (!(in && (in->flags & OR_TICK_NO_LOCALTICK))) local(e, r, OR_LOCAL_TICK);
  /* 4. proposals: tick input (synthetic Cmds of len P) or the batch staged by or_propose */
  uint32_t pn = 0;
  const ent_t* pents = NULL;
  const uint8_t* ppay = NULL;
  if (in && in->prop_target) {
    if (in->prop_target[r->g] == r->s) pn = in->prop_count[r->g];
  } else if (e->staged && e->stg_slot[r->g] == r->s) {
    pn = e->stg_n[r->g];
    pents = e->stg_ents + (size_t)r->g * e->c.max_entries_per_msg;
    ppay = e->stg_pay;
  }
  if (pn > 0) {
    msg_in_t mi;
    memset(&mi, 0, sizeof mi);
    mi.h.type = OR_PROPOSE;
    mi.h.from = (uint8_t)id_of(r->s);
    mi.h.nent = pn;
    mi.h.src_a = (uint32_t)(e->t % e->c.num_slabs);
    mi.h.src_b = 0;
    uint64_t hm = 0; /* entries with a non-empty Cmd */
    for (uint32_t k = 0; k < pn; ++k)
      if (e->c.payload_bytes && (!pents || pents[k].len)) hm |= 1ull << k;
    mi.h.hint = hm;
    mi.ents = pents;
    mi.pay = ppay;
    handle(e, r, &mi);
  }
  /* 4a. membership change input (or_config_change): one ConfigChange entry */
  if (e->cc_staged && e->cc_slot[r->g] == r->s) {
    msg_in_t mi;
    memset(&mi, 0, sizeof mi);
    mi.h.type = OR_PROPOSE;
    mi.h.from = (uint8_t)id_of(r->s);
    mi.h.nent = 1;
    mi.h.src_a = (uint32_t)(e->t % e->c.num_slabs);
    mi.h.hint_high = e->cc_desc[r->g];
    handle(e, r, &mi);
  }
  /* 4b. ReadIndex input */
  if (e->rd_staged && e->rd_req[rid]) {
    msg_in_t mi;
    memset(&mi, 0, sizeof mi);
    mi.h.type = OR_READ_INDEX;
    mi.h.from = (uint8_t)id_of(r->s);
    mi.h.hint = e->rd_req[rid];
    handle(e, r, &mi);
  }
  /* 5. apply + snapshot + compaction */
  /* GetUpdate.CommittedEntries = (processed, committed] (a restored range excluded), then
   * commitUpdate: processed = committed; applied follows unless the state machine reports it */
  r->apply_lo = u64max(processed_start, r->restored_at) + 1;
  /* the rsm applies the ConfigChange entries it is handed */
  for (uint64_t i = r->apply_lo; i <= r->committed; ++i) {
    const ent_t* en = log_at(e, r, i);
    if (en->type == OR_ENTRY_CONFIG && en->len) apply_config_change(e, r, en->len);
  }
  r->processed = r->committed;
  if (!e->c.apply_feedback) r->applied = r->processed;
  if (e->c.snapshot_entries && r->applied >= r->snap_index && r->applied - r->snap_index >= e->c.snapshot_entries) {
    r->snap_index = r->applied;
    r->snap_term = term_of(e, r, r->applied);
    r->snap_members = r->members;
    r->took = 1;
    uint64_t c = r->snap_index > e->c.compaction_overhead ? r->snap_index - e->c.compaction_overhead : 0;
    if (c > r->marker) {
      r->marker_term = term_of(e, r, c);
      r->marker = c;
    }
  }
  r->cap_base = marker_start;
  r->lpg = r->nlpg;
  r->fidx = r->marker != marker_start ? r->marker + 1 : 0;
}

typedef struct {
  or_engine* e;
  int w, T;
} worker_arg;

static void* worker(void* p) {
  worker_arg* a = (worker_arg*)p;
  or_engine* e = a->e;
  for (uint32_t g = (uint32_t)a->w; g < e->c.groups; g += (uint32_t)a->T)
    for (uint32_t s = 0; s < e->c.replicas; ++s) step_replica(e, &e->reps[g * e->c.replicas + s]);
  return NULL;
}

int or_tick(or_engine* e, const or_tick_input* in, int nthreads) {
  if (in && in->prop_target && e->staged) return -1; /* one proposal source per tick */
  e->in = in;
  if (nthreads <= 1) {
    worker_arg a = {e, 0, 1};
    worker(&a);
  } else {
    pthread_t th[256];
    worker_arg args[256];
    if (nthreads > 256) nthreads = 256;
    for (int w = 0; w < nthreads; ++w) {
      args[w].e = e;
      args[w].w = w;
      args[w].T = nthreads;
      pthread_create(&th[w], NULL, worker, &args[w]);
    }
    for (int w = 0; w < nthreads; ++w) pthread_join(th[w], NULL);
  }
  e->in = NULL;
  e->t++;
  if (e->staged) {
    memset(e->stg_slot, 0xFF, e->c.groups);
    memset(e->stg_n, 0, (size_t)e->c.groups * 4);
    e->stg_used = 0;
    e->staged = 0;
  }
  if (e->rd_staged) {
    memset(e->rd_req, 0, (size_t)e->nrep * 8);
    e->rd_staged = 0;
  }
  if (e->cc_staged) {
    memset(e->cc_slot, 0xFF, e->c.groups);
    e->cc_staged = 0;
  }
  return 0;
}

int or_config_change(or_engine* e, uint64_t group, uint32_t slot, uint32_t op, uint32_t target) {
  if (group < e->c.group_base || group >= (uint64_t)e->c.group_base + e->c.groups || slot >= e->c.replicas ||
      target >= e->c.replicas || (op != OR_CC_ADD && op != OR_CC_REMOVE))
    return -1;
  uint32_t g = (uint32_t)(group - e->c.group_base);
  if (e->cc_slot[g] != 0xFF) return -3;
  e->cc_slot[g] = (uint8_t)slot;
  e->cc_desc[g] = (uint8_t)OR_CC(op, target);
  e->cc_staged = 1;
  return 0;
}

int or_compact(or_engine* e, uint64_t group, uint64_t index) {
  if (group < e->c.group_base || group >= (uint64_t)e->c.group_base + e->c.groups) return -1;
  const uint32_t g = (uint32_t)(group - e->c.group_base);
  int n = 0;
  for (uint32_t s = 0; s < e->c.replicas; ++s) {
    rep_t* r = &e->reps[g * e->c.replicas + s];
    const uint64_t c = index < r->snap_index ? index : r->snap_index;
    if (c <= r->marker) continue;
    r->marker_term = term_of(e, r, c);
    r->marker = c;
    r->fidx = c + 1; /* the next step releases the stream below entry c + 1 */
    ++n;
  }
  return n;
}

int or_read_index(or_engine* e, const or_read_request* q, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if (q[i].group < e->c.group_base || q[i].group >= (uint64_t)e->c.group_base + e->c.groups ||
        q[i].slot >= e->c.replicas || q[i].ctx == 0)
      return -1;
  for (size_t i = 0; i < n; ++i) e->rd_req[(q[i].group - e->c.group_base) * e->c.replicas + q[i].slot] = q[i].ctx;
  if (n) e->rd_staged = 1;
  return 0;
}

int or_get_read_ready(const or_engine* e, uint32_t rid, uint64_t* ctx, uint64_t* index, uint32_t cap) {
  if (rid >= e->nrep) return -1;
  const rep_t* r = &e->reps[rid];
  if (r->rd_tick != e->t) return 0; /* none made ready in the last step */
  for (uint32_t i = 0; i < r->rd_n && i < cap; ++i) {
    if (ctx) ctx[i] = r->rd_ctx[i];
    if (index) index[i] = r->rd_index[i];
  }
  return (int)r->rd_n;
}

int or_propose(or_engine* e, const or_proposal* p, size_t n, const uint8_t* payload, const uint32_t* lens) {
  const uint32_t G = e->c.groups, E = e->c.max_entries_per_msg, P = e->c.payload_bytes;
  uint64_t tot = 0;
  for (size_t i = 0; i < n; ++i) tot = p[i].first + p[i].count > tot ? p[i].first + p[i].count : tot;
  /* byte offset of every entry: Cmds packed in lens order */
  uint64_t* off = (uint64_t*)calloc(tot + 1, 8);
  for (uint64_t j = 0; j < tot; ++j) off[j + 1] = off[j] + (lens ? lens[j] : 0);
  /* validate everything before staging anything */
  uint8_t* slot = (uint8_t*)malloc(G);
  uint32_t* cnt = (uint32_t*)malloc((size_t)G * 4);
  memcpy(slot, e->stg_slot, G);
  memcpy(cnt, e->stg_n, (size_t)G * 4);
  int rc = 0;
  for (size_t i = 0; i < n && !rc; ++i) {
    if (p[i].group < e->c.group_base || p[i].group >= (uint64_t)e->c.group_base + G || p[i].slot >= e->c.replicas ||
        p[i].count < 1 || p[i].count > E) {
      rc = -1;
      break;
    }
    for (uint64_t j = p[i].first; j < p[i].first + p[i].count; ++j)
      if (lens && lens[j] > e->maxc) rc = -1;
    uint32_t g = (uint32_t)(p[i].group - e->c.group_base);
    if (!rc && cnt[g] && slot[g] != p[i].slot) rc = -3;
    if (!rc && cnt[g] + p[i].count > E) rc = -3;
    if (!rc) {
      slot[g] = (uint8_t)p[i].slot;
      cnt[g] += p[i].count;
    }
  }
  if (!rc) {
    for (size_t i = 0; i < n; ++i) {
      uint32_t g = (uint32_t)(p[i].group - e->c.group_base);
      e->stg_slot[g] = (uint8_t)p[i].slot;
      for (uint32_t k = 0; k < p[i].count; ++k) {
        uint64_t j = p[i].first + k, at = (uint64_t)g * E + e->stg_n[g] + k;
        uint32_t len = lens ? lens[j] : 0;
        e->stg_ents[at].len = len;
        e->stg_ents[at].off = 0;
        if (P && len) {
          e->stg_ents[at].off = bytes_reserve(&e->stg_pay, &e->stg_used, &e->stg_cap, len);
          memcpy(e->stg_pay + e->stg_ents[at].off, payload + off[j], len);
        }
      }
      e->stg_n[g] += p[i].count;
    }
    e->staged = n > 0 || e->staged;
  }
  free(slot);
  free(cnt);
  free(off);
  return rc;
}

/* ---------------------------------------------------------------- lifecycle / views */

int or_create(const or_config* cfg, or_engine** out) {
  const or_config* c = cfg;
  if (c->replicas < 1 || c->replicas > OR_MAX_R) return -1;
  if (c->log_capacity < 16 || (c->log_capacity & (c->log_capacity - 1))) return -1;
  if (c->payload_bytes && (c->payload_bytes < 16 || c->payload_bytes > 1024 ||
                           (c->payload_bytes & (c->payload_bytes - 1))))
    return -1;
  if (c->max_entries_per_msg < 1 || c->max_entries_per_msg > 64) return -1;
  if (c->max_msgs_per_pair < 1 || c->max_msgs_per_pair > 16) return -1;
  if (c->num_slabs < 2 || c->election_rtt < 1 || c->heartbeat_rtt < 1) return -1;
  if (c->initial_members >> c->replicas) return -1;
  if (c->join_slots >> c->replicas || (c->initial_members & c->join_slots)) return -1;
  uint32_t maxc = c->max_cmd_bytes ? c->max_cmd_bytes : c->payload_bytes;
  if (c->payload_bytes ? (maxc < c->payload_bytes || maxc > OR_MAX_CMD) : maxc != 0) return -1;
  or_engine* e = (or_engine*)calloc(1, sizeof *e);
  e->c = *c;
  e->nrep = c->groups * c->replicas;
  e->maxc = maxc;
  { /* stream_pages as rg_create sizes it: twice a full log of P-byte Cmds, plus two of the longest */
    uint64_t full = ((uint64_t)c->log_capacity * ((c->payload_bytes + 15) & ~15u) + 4095) / 4096;
    uint64_t big = maxc > c->payload_bytes ? 2 * (((uint64_t)maxc + 4095) / 4096 + 1) : 0;
    uint32_t pts = 16;
    while (pts < 2 * full + big) pts <<= 1;
    e->pts = c->payload_bytes ? (c->stream_pages ? c->stream_pages : pts) : 1;
  }
  e->stg_slot = (uint8_t*)malloc(c->groups);
  memset(e->stg_slot, 0xFF, c->groups);
  e->stg_n = (uint32_t*)calloc(c->groups, 4);
  e->stg_ents = (ent_t*)calloc((size_t)c->groups * c->max_entries_per_msg, sizeof(ent_t));
  e->stg_pay = NULL;
  e->stg_used = e->stg_cap = 0;
  e->rd_req = (uint64_t*)calloc((size_t)c->groups * c->replicas, 8);
  e->cc_slot = (uint8_t*)malloc(c->groups);
  memset(e->cc_slot, 0xFF, c->groups);
  e->cc_desc = (uint8_t*)calloc(c->groups, 1);
  e->reps = (rep_t*)calloc(e->nrep, sizeof(rep_t));
  for (uint32_t i = 0; i < e->nrep; ++i) {
    rep_t* r = &e->reps[i];
    r->g = i / c->replicas;
    r->s = i % c->replicas;
    r->log = (ent_t*)calloc(c->log_capacity, sizeof(ent_t));
    r->cmd = (uint8_t**)calloc(c->log_capacity, sizeof(uint8_t*));
    r->cmdcap = (uint32_t*)calloc(c->log_capacity, 4);
    /* pre-fault the ring so timed ticks do not pay first-touch page faults (and give every slot room
     * for a P-byte Cmd, the benchmark's) */
    memset(r->log, 0, (size_t)c->log_capacity * sizeof(ent_t));
    if (c->payload_bytes)
      for (uint32_t k = 0; k < c->log_capacity; ++k) {
        r->cmd[k] = (uint8_t*)calloc(c->payload_bytes, 1);
        r->cmdcap[k] = c->payload_bytes;
      }
    for (int b = 0; b < 2; ++b)
      r->ob[b].m = (msg_t*)calloc((size_t)c->replicas * c->max_msgs_per_pair, sizeof(msg_t));
  }
  *out = e;
  return 0;
}

void or_destroy(or_engine* e) {
  if (!e) return;
  for (uint32_t i = 0; i < e->nrep; ++i) {
    rep_t* r = &e->reps[i];
    free(r->log);
    if (r->cmd)
      for (uint32_t k = 0; k < e->c.log_capacity; ++k) free(r->cmd[k]);
    free(r->cmd);
    free(r->cmdcap);
    for (int b = 0; b < 2; ++b) {
      free(r->ob[b].m);
      free(r->ob[b].ents);
      free(r->ob[b].pay);
    }
  }
  free(e->reps);
  free(e->stg_slot);
  free(e->stg_n);
  free(e->stg_ents);
  free(e->stg_pay);
  free(e->rd_req);
  free(e->cc_slot);
  free(e->cc_desc);
  free(e);
}

/* peer.go Launch(newNode) → becomeFollower(1, NoLeader); bootstrap(addresses) (A.2) */
/* A joining replica (join_slots; StartOnDiskReplica with join = true, raft/raft_manager.go:134-144)
 * starts with an empty log at term 0 and no membership: becomeFollower(0, NoLeader). The others
 * bootstrap with one ConfigChange entry per slot at term 1 — AddNode(s) for each initial member,
 * descriptor 0 for the other slots — committed. */
int or_bootstrap(or_engine* e) {
  uint32_t R = e->c.replicas;
  uint32_t im = (e->c.initial_members ? e->c.initial_members : (1u << R) - 1u) & ~e->c.join_slots;
  for (uint32_t i = 0; i < e->nrep; ++i) {
    rep_t* r = &e->reps[i];
    int joining = (e->c.join_slots >> r->s) & 1u;
    r->term = 0;
    r->last = r->marker = r->marker_term = r->committed = r->applied = r->processed = 0;
    r->snap_index = r->snap_term = r->cap_base = 0;
    r->err = r->drops = 0;
    r->rng_ctr = 0;
    r->hw = r->lpg = r->nlpg = 0;
    r->fidx = 0;
    r->members = r->snap_members = joining ? 0u : im;
    become_follower(e, r, joining ? 0 : 1, 0);
    uint32_t last = joining ? 0 : R;
    for (uint32_t k = 0; k < last; ++k) {
      ent_t* en = log_at(e, r, k + 1);
      en->term = 1;
      en->type = OR_ENTRY_CONFIG;
      en->len = ((im >> k) & 1u) ? OR_CC(OR_CC_ADD, k) : 0u;
      en->crc = 0;
      en->pos = 0;
    }
    r->last = last;
    r->committed = last;
    for (uint32_t k = 0; k < R; ++k) { /* addNode → setRemote(id, 0, last+1) */
      r->match[k] = 0;
      r->next[k] = last + 1;
      r->rsnap[k] = 0;
      r->rstate[k] = OR_RETRY;
    }
    for (int b = 0; b < 2; ++b) {
      memset(r->ob[b].n, 0, sizeof r->ob[b].n);
      r->ob[b].n_ents = 0;
      r->ob[b].pay_used = 0;
    }
  }
  e->t = 0;
  return 0;
}

uint64_t or_tick_count(const or_engine* e) { return e->t; }

int or_get_replica(const or_engine* e, uint32_t rid, or_replica_view* v) {
  if (rid >= e->nrep) return -1;
  const rep_t* r = &e->reps[rid];
  memset(v, 0, sizeof *v);
  v->term = r->term;
  v->vote = r->vote;
  v->leader = r->leader;
  v->committed = r->committed;
  v->applied = r->applied;
  v->processed = r->processed;
  v->last = r->last;
  v->marker = r->marker;
  v->marker_term = r->marker_term;
  v->snap_index = r->snap_index;
  v->snap_term = r->snap_term;
  v->cap_base = r->cap_base;
  v->role = r->role;
  v->election_tick = r->election_tick;
  v->heartbeat_tick = r->heartbeat_tick;
  v->rand_timeout = r->rand_timeout;
  v->rng_ctr = r->rng_ctr;
  v->granted = r->granted;
  v->responded = r->responded;
  v->active = r->active;
  v->err = r->err;
  v->drops = r->drops;
  v->members = r->members;
  v->snap_members = r->snap_members;
  v->cc_pending = r->cc_pending;
  for (uint32_t k = 0; k < e->c.replicas; ++k) {
    v->match[k] = r->match[k];
    v->next[k] = r->next[k];
    v->rsnap[k] = r->rsnap[k];
    v->rstate[k] = r->rstate[k];
  }
  return 0;
}

int or_get_replicas(const or_engine* e, uint32_t first, uint32_t n, or_replica_view* out) {
  if ((uint64_t)first + n > e->nrep) return -1;
  for (uint32_t i = 0; i < n; ++i) or_get_replica(e, first + i, &out[i]);
  return 0;
}

static const outbox_t* last_ob(const or_engine* e, const rep_t* r) { return &r->ob[(e->t + 1) & 1]; }

int or_get_msgs(const or_engine* e, uint32_t rid, uint32_t dst, or_msg_view* out, uint32_t cap) {
  if (rid >= e->nrep || dst >= e->c.replicas) return -1;
  const outbox_t* ob = last_ob(e, &e->reps[rid]);
  uint32_t n = ob->n[dst];
  for (uint32_t k = 0; k < n && k < cap; ++k) out[k] = ob->m[dst * e->c.max_msgs_per_pair + k].h;
  return (int)n;
}

int or_get_msg_terms(const or_engine* e, uint32_t rid, uint32_t dst, uint32_t k, uint64_t* terms, uint32_t cap) {
  if (rid >= e->nrep || dst >= e->c.replicas) return -1;
  const outbox_t* ob = last_ob(e, &e->reps[rid]);
  if (k >= ob->n[dst]) return -1;
  const msg_t* m = &ob->m[dst * e->c.max_msgs_per_pair + k];
  uint32_t n = m->h.type == OR_REPLICATE ? m->h.nent : 0;
  for (uint32_t i = 0; i < n && i < cap; ++i) terms[i] = ob->ents[m->ent_off + i].term;
  return (int)n;
}

int or_get_entry(const or_engine* e, uint32_t rid, uint64_t index, or_entry_view* out, uint8_t* payload) {
  if (rid >= e->nrep) return -1;
  const rep_t* r = &e->reps[rid];
  if (index <= r->marker || index > r->last) return -1;
  const ent_t* en = log_at(e, r, index);
  out->term = en->term;
  out->type = en->type;
  out->len = en->len;
  out->crc = en->crc;
  out->_pad = 0;
  if (payload && en->len && en->type == OR_ENTRY_APP) memcpy(payload, logpay_at(e, r, index), en->len);
  return 0;
}

int or_import_replica(or_engine* e, uint32_t rid, const or_replica_view* v, const uint64_t* terms,
                      const uint32_t* types, const uint8_t* payloads, const uint32_t* lens) {
  if (rid >= e->nrep) return -1;
  rep_t* r = &e->reps[rid];
  if (v->last < v->marker || v->last - v->marker > e->c.log_capacity) return -1;
  if (lens)
    for (uint64_t k = 0; k < v->last - v->marker; ++k)
      if (lens[k] > e->maxc && !(types && (types[k] & 0xFFu) == OR_ENTRY_CONFIG)) return -1;
  r->term = v->term;
  r->vote = v->vote;
  r->leader = v->leader;
  r->committed = v->committed;
  r->applied = v->applied;
  r->processed = v->processed;
  r->last = v->last;
  r->marker = v->marker;
  r->marker_term = v->marker_term;
  r->snap_index = v->snap_index;
  r->snap_term = v->snap_term;
  r->cap_base = v->cap_base;
  r->restored_at = 0;
  r->apply_lo = v->processed + 1; /* nothing to apply until it steps */
  r->took = 0;
  r->rq_n = 0;
  r->rd_tick = 0;
  r->role = v->role;
  r->election_tick = v->election_tick;
  r->heartbeat_tick = v->heartbeat_tick;
  r->rand_timeout = v->rand_timeout;
  r->rng_ctr = v->rng_ctr;
  r->granted = v->granted;
  r->responded = v->responded;
  r->active = v->active;
  r->err = v->err;
  r->drops = v->drops;
  r->members = v->members;
  r->snap_members = v->snap_members;
  r->cc_pending = v->cc_pending;
  for (uint32_t k = 0; k < OR_MAX_R; ++k) {
    r->match[k] = v->match[k];
    r->next[k] = v->next[k];
    r->rsnap[k] = v->rsnap[k];
    r->rstate[k] = v->rstate[k];
  }
  uint32_t P = e->c.payload_bytes;
  r->hw = r->lpg = r->nlpg = 0; /* a fresh payload stream (rg_import_replica) */
  r->fidx = 0;
  uint64_t src = 0; /* the Cmds come packed back to back, one per entry that has one */
  for (uint64_t i = v->marker + 1; i <= v->last; ++i) {
    uint64_t k = i - v->marker - 1;
    ent_t* en = log_at(e, r, i);
    en->term = terms[k];
    en->type = types ? (types[k] & 0xFFu) : OR_ENTRY_APP;
    en->pos = r->hw;
    uint32_t len = lens ? lens[k] : P;
    if (payloads && P && len && en->type == OR_ENTRY_APP && !(types && (types[k] & OR_ENTRY_EMPTY))) {
      en->len = len;
      uint8_t* d = logpay_put(e, r, i, len);
      memcpy(d, payloads + src, len);
      src += len;
      en->crc = entry_crc(e, d, len);
      r->hw += chunks_of(len);
    } else {
      en->len = en->type == OR_ENTRY_CONFIG && lens ? lens[k] : 0; /* a ConfigChange keeps its descriptor */
      en->crc = 0;
    }
  }
  r->lpg = r->nlpg = 0;
  return 0;
}

int or_deliver(or_engine* e, uint32_t rid_src, const or_msg_view* m) {
  if (rid_src >= e->nrep) return -1;
  rep_t* r = &e->reps[rid_src];
  outbox_t* ob = &r->ob[(e->t + 1) & 1];
  uint32_t dst = slot_of(m->to);
  if (dst >= e->c.replicas || ob->n[dst] >= e->c.max_msgs_per_pair) return -1;
  msg_t* mm = &ob->m[dst * e->c.max_msgs_per_pair + ob->n[dst]++];
  mm->h = *m;
  mm->ent_off = 0;
  if (m->type == OR_REPLICATE && m->nent) {
    if (m->log_index < r->marker || m->log_index + m->nent > r->last) return -1;
    arena_reserve(e, ob, m->nent);
    mm->ent_off = (uint32_t)ob->n_ents;
    for (uint32_t k = 0; k < m->nent; ++k) {
      ent_t* en = &ob->ents[ob->n_ents + k];
      *en = *log_at(e, r, m->log_index + 1 + k);
      if (e->c.payload_bytes) ob_put_cmd(ob, en, logpay_at(e, r, m->log_index + 1 + k));
    }
    ob->n_ents += m->nent;
  }
  return 0;
}

int or_notify_applied(or_engine* e, uint32_t rid, uint64_t index) {
  if (rid >= e->nrep) return -1;
  rep_t* r = &e->reps[rid];
  if (index > r->processed) return -1;
  r->applied = index;
  return 0;
}

/* Snapshot events of replica rid's last step (rg_snapshot_events): returns OR_SNAP_* bits;
 * restored = the index an InstallSnapshot restored the log to, index/term = the snapshot taken. */
/* the first index replica rid's last step handed to the state machine (its apply window starts
 * there; tests compare the engine's hand-off word with it) */
int or_debug_apply_lo(const or_engine* e, uint32_t rid, uint64_t* apply_lo) {
  if (rid >= e->nrep || !apply_lo) return -1;
  *apply_lo = e->reps[rid].apply_lo;
  return 0;
}

int or_get_snapshot_event(const or_engine* e, uint32_t rid, uint64_t* restored, uint64_t* index, uint64_t* term) {
  if (rid >= e->nrep) return -1;
  const rep_t* r = &e->reps[rid];
  if (restored) *restored = r->restored_at;
  if (index) *index = r->took ? r->snap_index : 0;
  if (term) *term = r->took ? r->snap_term : 0;
  return (r->restored_at ? OR_SNAP_RESTORED : 0) | (r->took ? OR_SNAP_TAKEN : 0);
}

/* The non-empty application entries replica rid handed to the state machine in the last step
 * (dragonboat's rsm skips config changes and empty entries before Update), read from the log ring
 * where they stay until the next step may reuse their slots (capacity rule). */
int or_get_applied(const or_engine* e, uint32_t rid, uint64_t* index, or_entry_view* out, uint8_t* payload,
                   uint32_t cap) {
  if (rid >= e->nrep) return -1;
  const rep_t* r = &e->reps[rid];
  uint32_t n = 0;
  uint64_t at = 0; /* payload: the Cmds packed back to back */
  for (uint64_t i = r->apply_lo ? r->apply_lo : 1; i <= r->processed; ++i) {
    const ent_t* en = log_at(e, r, i);
    if (en->type != OR_ENTRY_APP || en->len == 0) continue;
    if (n < cap) {
      if (index) index[n] = i;
      if (out) {
        out[n].term = en->term;
        out[n].type = en->type;
        out[n].len = en->len;
        out[n].crc = en->crc;
        out[n]._pad = 0;
      }
      if (payload && e->c.payload_bytes) {
        memcpy(payload + at, logpay_at(e, r, i), en->len);
        at += en->len;
      }
    }
    n++;
  }
  return (int)n;
}

/* ---- whole-table digest (or_digest, oracle.h; rg_digest restates it on the device) */
static inline uint64_t dg_mix(uint64_t z) {  /* fmix64 */
  z ^= z >> 33;
  z *= 0xFF51AFD7ED558CCDULL;
  z ^= z >> 33;
  z *= 0xC4CEB9FE1A85EC53ULL;
  z ^= z >> 33;
  return z;
}

int or_digest(const or_engine* e, uint64_t out[2]) {
  uint64_t a = 0, b = 0;
  const uint32_t R = e->c.replicas;
  for (uint32_t rid = 0; rid < e->nrep; ++rid) {
    const rep_t* r = &e->reps[rid];
    or_replica_view v;
    or_get_replica(e, rid, &v);
    const uint64_t gid = global_group(e, r) * R + r->s;
    uint64_t h = dg_mix(gid + 0x9E3779B97F4A7C15ULL);
    const uint64_t f[25] = {v.term, v.vote, v.leader, v.committed, v.applied, v.last, v.marker, v.marker_term,
                            v.snap_index, v.snap_term, v.cap_base, v.processed, v.role, v.election_tick,
                            v.heartbeat_tick, v.rand_timeout, v.rng_ctr, v.granted, v.responded, v.active, v.err,
                            v.drops, v.members, v.snap_members, v.cc_pending};
    for (int k = 0; k < 25; ++k) h = dg_mix(h ^ f[k]);
    for (uint32_t j = 0; j < R; ++j) {
      h = dg_mix(h ^ v.match[j]);
      h = dg_mix(h ^ v.next[j]);
      h = dg_mix(h ^ v.rsnap[j]);
      h = dg_mix(h ^ v.rstate[j]);
    }
    a += h;
    uint64_t h2 = dg_mix(gid ^ 0x5851F42D4C957F2DULL);
    for (uint64_t i = r->marker + 1; i <= r->last; ++i) {
      const ent_t* en = log_at(e, r, i);
      h2 = dg_mix(h2 ^ en->term);
      h2 = dg_mix(h2 ^ ((uint64_t)en->type | ((uint64_t)en->len << 8) | ((uint64_t)en->crc << 32)));
    }
    b += h2;
  }
  out[0] = a;
  out[1] = b;
  return 0;
}
