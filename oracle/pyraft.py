"""Independent pure-Python restatement of the per-shard Raft step.

TEST INFRASTRUCTURE. Written separately from oracle/oracle.c (different structure: objects,
dict messages, Python lists as logs) so that tick-by-tick agreement between the two on random
seeded traces is evidence that the restatement says what DESIGN.md §1 says. It restates
dragonboat v4 internal/raft (module github.com/lni/dragonboat/v4
v4.0.0-20240618143154-6a1623140f27, absent here: parity with dragonboat itself is unpinned)
following SURVEY.md Appendix A:
  A.3 Handle / onMessageTermNotMatched   -> Replica.handle
  A.5 reset / become*                    -> Replica.reset / become_*
  A.6 leaderTick / nonLeaderTick         -> Replica.tick
  A.7 campaign                           -> Replica.campaign
  A.8 handleNodeRequestVote / VoteResp   -> Replica.on_request_vote / on_vote_resp
  A.9 handleReplicateMessage             -> Replica.on_replicate
  A.10 handleLeaderReplicateResp         -> Replica.on_replicate_resp
  A.11 handleLeaderHeartbeatResp         -> Replica.on_heartbeat_resp
  A.12 sendReplicateMessage              -> Replica.send_replicate
  A.13 tryCommit                         -> Replica.try_commit
Only for small configurations (it is slow).
"""
from __future__ import annotations

import zlib

M64 = (1 << 64) - 1

LOCAL_TICK, ELECTION, LEADER_HEARTBEAT, NOOP, PROPOSE = 0, 1, 2, 4, 7
CHECK_QUORUM, REPLICATE, REPLICATE_RESP, REQUEST_VOTE, REQUEST_VOTE_RESP = 10, 12, 13, 14, 15
INSTALL_SNAPSHOT, HEARTBEAT, HEARTBEAT_RESP = 16, 17, 18
READ_INDEX, READ_INDEX_RESP = 19, 20
FOLLOWER, CANDIDATE, LEADER = 0, 1, 2
RETRY, WAIT, REPL, SNAP = 0, 1, 2, 3
ERR_CONFLICT, ERR_BEYOND, ERR_RING, ERR_CRC, ERR_EMPTY_SNAP = 1, 2, 4, 8, 16
ERR_TERM = 128  # a campaign at the last term the ring word holds (2^36 - 1): refused
TERM_MAX = (1 << 36) - 1
RQ = 4  # ReadIndex requests a leader holds pending, reads a replica makes ready per step
LEADER_MSGS = (REPLICATE, INSTALL_SNAPSHOT, HEARTBEAT, READ_INDEX_RESP)
CC_ADD, CC_REMOVE = 1, 2  # membership change ops: descriptor op << 4 | (slot + 1)


def mix64(z: int) -> int:
    z &= M64
    z ^= z >> 30
    z = (z * 0xBF58476D1CE4E5B9) & M64
    z ^= z >> 27
    z = (z * 0x94D049BB133111EB) & M64
    z ^= z >> 31
    return z


def payload(seed: int, slab: int, group: int, entry: int, P: int) -> bytes:
    key = mix64(((slab << 56) ^ (group << 16) ^ entry ^ ((seed * 0x9E3779B97F4A7C15) & M64)) & M64)
    out = bytearray()
    for w in range(P // 8):
        out += mix64((key + (w + 1) * 0xD1B54A32D192ED03) & M64).to_bytes(8, "little")
    return bytes(out)


def msg(type, to, **kw):
    m = dict(type=type, to=to, frm=0, reject=0, nent=0, term=0, log_term=0, log_index=0, commit=0,
             hint=0, hint_high=0, src_a=0, src_b=0, ents=())
    m.update(kw)
    return m


class Entry:
    __slots__ = ("term", "type", "data", "crc", "cc", "pos")

    def __init__(self, term, type=0, data=b"", cc=0):
        self.term, self.type, self.data, self.cc = term, type, data, cc
        self.crc = zlib.crc32(data) if data else 0
        self.pos = 0  # payload stream position (16-B chunks) in the log that holds it

    @property
    def chunks(self):
        return (len(self.data) + 15) // 16 if self.type == 0 else 0

    @property
    def len(self):
        """Cmd length; a ConfigChange entry reports its descriptor."""
        return self.cc if self.type == 1 else len(self.data)


class Remote:
    __slots__ = ("match", "next", "snap", "state")

    def __init__(self, match, nxt):
        self.match, self.next, self.snap, self.state = match, nxt, 0, RETRY

    # remote.go
    def try_update(self, idx):
        if self.next < idx + 1:
            self.next = idx + 1
        if self.match < idx:
            if self.state == WAIT:
                self.state = RETRY
            self.match = idx
            return True
        return False

    def become_retry(self):
        self.next = max(self.match + 1, self.snap + 1) if self.state == SNAP else self.match + 1
        self.snap = 0
        self.state = RETRY

    def responded_to(self):
        if self.state == RETRY:
            self.next, self.snap, self.state = self.match + 1, 0, REPL
        elif self.state == SNAP and self.match >= self.snap:
            self.become_retry()

    def decrease_to(self, rejected, last):
        if self.state == REPL:
            if rejected <= self.match:
                return False
            self.next = self.match + 1
            return True
        if self.next - 1 != rejected:
            return False
        if self.state == WAIT:
            self.state = RETRY
        self.next = max(1, min(rejected, last + 1))
        return True

    def progress(self, last_sent):
        if self.state == REPL:
            self.next = last_sent + 1
        elif self.state == RETRY:
            self.state = WAIT

    def paused(self):
        return self.state in (WAIT, SNAP)


class Replica:
    def __init__(self, sim, g, s):
        self.sim, self.g, self.s, self.id = sim, g, s, s + 1
        self.term = self.vote = self.leader = 0
        self.role = FOLLOWER
        self.committed = self.applied = self.processed = 0
        self.marker = self.marker_term = 0
        self.log = []  # log[k] = entry at index marker+1+k
        self.snap_index = self.snap_term = self.cap_base = 0
        self.etick = self.htick = self.rand_to = self.rng = 0
        self.votes = {}
        self.active = set()
        self.err = self.drops = 0
        self.remotes = []
        self.out = {}
        self.emitted = {}
        self.pending_reads = []  # leader, arrival order: [ctx, index, acks set, requester slot]
        self.ready_reads = None  # (tick, [(ctx, index), ...]) of the reads made ready in a step
        self.members = set(range(sim.R))  # voting membership as applied here
        self.snap_members = set(range(sim.R))
        self.cc_pending = False
        self.restored_at = 0
        # payload stream: next free chunk, lowest page held, the last step's compaction bound
        self.hw = self.lpg = self.nlpg = self.fidx = 0

    @property
    def quorum(self):
        return len(self.members) // 2 + 1

    # -- log (entryLog) --
    @property
    def last(self):
        return self.marker + len(self.log)

    def term_at(self, i):
        if i == self.marker:
            return self.marker_term
        if self.marker < i <= self.last:
            return self.log[i - self.marker - 1].term
        return 0

    def up_to_date(self, i, t):
        lt = self.term_at(self.last)
        return t > lt or (t == lt and i >= self.last)

    def stream_fits(self, chunks):
        """The stream capacity rule: the append's last chunk within stream_pages of the lowest page held."""
        if chunks == 0:
            return True
        return (((self.hw + chunks - 1) & 0xFFFFFFFF) >> 8) - self.lpg & 0xFFFFFF < self.sim.pts

    def put(self, e):
        """Append Entry e to the log at the stream's end."""
        e.pos = self.hw
        self.hw = (self.hw + e.chunks) & 0xFFFFFFFF
        self.log.append(e)

    def commit_to(self, i):
        if i <= self.committed:
            return
        if i > self.last:
            self.err |= ERR_BEYOND
            return
        self.committed = i

    # -- transport --
    def send(self, m):
        c = self.sim.cfg
        m["frm"] = self.id
        if m["type"] not in (PROPOSE, REQUEST_VOTE, READ_INDEX):
            m["term"] = self.term
        d = m["to"] - 1
        n = self.emitted.get(d, 0)
        self.emitted[d] = n + 1
        if self.sim.lost(self, d, n) or len(self.out.setdefault(d, [])) >= c["max_msgs_per_pair"]:
            self.drops += 1
            return False
        self.out[d].append(m)
        return True

    # -- transitions --
    def reset(self, t):
        if t != self.term:
            self.term, self.vote = t, 0
        self.leader = 0
        self.votes = {}
        self.etick = self.htick = 0
        self.rng += 1
        c = self.sim.cfg
        key = (self.g << 32) | (self.s << 24) | (self.rng & 0xFFFFFF)
        self.rand_to = c["election_rtt"] + mix64(c["seed"] ^ mix64(key)) % c["election_rtt"]
        self.remotes = [Remote(0, self.last + 1) for _ in range(self.sim.R)]
        self.remotes[self.s].match = self.last
        self.active = set()
        self.pending_reads = []  # readIndex.reset
        self.cc_pending = False  # clearPendingConfigChange

    def become_follower(self, t, leader):
        self.role = FOLLOWER
        self.reset(t)
        self.leader = leader

    def become_candidate(self):
        self.role = CANDIDATE
        self.reset(self.term + 1)
        self.leader = 0
        self.vote = self.id

    def become_leader(self):
        self.role = LEADER
        self.reset(self.term)
        self.leader = self.id
        # a ConfigChange entry not yet committed is still in flight
        self.cc_pending = any(self.log[i - self.marker - 1].type == 1 for i in range(self.committed + 1, self.last + 1))
        if not self.append(1, ()):
            self.err |= ERR_RING

    def append(self, n, cmds, cc=0):
        """appendEntries of n entries at the current term; cmds[k] = Cmd bytes of entry k (() for
        the leader's empty no-op); cc: one ConfigChange entry with that descriptor."""
        c = self.sim.cfg
        if self.last + n > self.cap_base + c["log_capacity"]:
            return False
        if not cc and not self.stream_fits(sum((len(x) + 15) // 16 for x in cmds[:n])):
            return False
        for k in range(n):
            if cc:
                self.put(Entry(self.term, 1, b"", cc))
            else:
                self.put(Entry(self.term, 0, cmds[k] if k < len(cmds) else b""))
        self.remotes[self.s].try_update(self.last)
        if len(self.members) == 1:
            self.try_commit()
        return True

    # -- leader --
    def try_commit(self):
        vals = sorted(self.remotes[i].match for i in self.members)
        if not vals:
            return False
        q = vals[len(vals) - self.quorum]
        if q > self.committed and self.term_at(q) == self.term:
            self.committed = q
            return True
        return False

    def send_replicate(self, to):
        rp = self.remotes[to]
        if rp.paused():
            return
        if rp.next <= self.marker:
            if to not in self.active:
                return
            if self.snap_index == 0:
                self.err |= ERR_EMPTY_SNAP
                return
            rp.snap, rp.state = self.snap_index, SNAP
            self.send(msg(INSTALL_SNAPSHOT, to + 1, log_index=self.snap_index, log_term=self.snap_term,
                          hint_high=sum(1 << k for k in self.snap_members)))
            return
        nxt = rp.next
        ents = self.log[nxt - self.marker - 1: nxt - self.marker - 1 + self.sim.cfg["max_entries_per_msg"]] \
            if nxt <= self.last else []
        if ents:
            rp.progress(nxt + len(ents) - 1)
        self.send(msg(REPLICATE, to + 1, log_index=nxt - 1, log_term=self.term_at(nxt - 1),
                      commit=self.committed, nent=len(ents), ents=tuple(ents)))

    def broadcast_replicate(self):
        for i in range(self.sim.R):
            if i != self.s and i in self.members:
                self.send_replicate(i)

    def on_replicate_resp(self, m):
        f = m["frm"] - 1
        if f not in self.members:
            return
        rp = self.remotes[f]
        self.active.add(f)
        if not m["reject"]:
            was_paused = rp.paused()
            if rp.try_update(m["log_index"]):
                rp.responded_to()
                if self.try_commit():
                    self.broadcast_replicate()
                elif was_paused:
                    self.send_replicate(f)
        elif rp.decrease_to(m["log_index"], m["hint"]):
            if rp.state == REPL:
                rp.become_retry()
            self.send_replicate(f)

    def on_heartbeat_resp(self, m):
        f = m["frm"] - 1
        if f not in self.members:
            return
        self.active.add(f)
        rp = self.remotes[f]
        if rp.state == WAIT:
            rp.state = RETRY
        if rp.match < self.last:
            self.send_replicate(f)
        # readIndex.confirm: once a quorum confirmed the answered request, it and every request queued
        # before it are done, all at its index
        q = self.pending_reads
        k = next((i for i, pr in enumerate(q) if pr[0] == m["hint"]), None) if m["hint"] else None
        if k is not None:
            q[k][2].add(f)
            if len(q[k][2] & self.members) >= self.quorum:
                done, self.pending_reads = q[:k + 1], q[k + 1:]
                for ctx, _, _, slot in done:
                    self.read_confirmed(ctx, q[k][1], slot)

    # -- ReadIndex (Raft thesis §6.4; dragonboat's readIndex queue) --
    def read_ready_add(self, ctx, index):  # addReadyToRead, at most RQ per step
        if self.ready_reads is None or self.ready_reads[0] != self.sim.t:
            self.ready_reads = (self.sim.t, [])
        if len(self.ready_reads[1]) == RQ:
            self.drops += 1
        else:
            self.ready_reads[1].append((ctx, index))

    def read_confirmed(self, ctx, index, slot):
        if slot == self.s:
            self.read_ready_add(ctx, index)
        else:
            self.send(msg(READ_INDEX_RESP, slot + 1, log_index=index, hint=ctx))

    def on_read_index(self, m):
        f = m["frm"] - 1
        if self.role == LEADER:
            if self.quorum == 1:
                self.read_confirmed(m["hint"], self.committed, f)
            elif self.term_at(self.committed) != self.term:
                self.drops += 1
            else:
                if all(pr[0] != m["hint"] for pr in self.pending_reads):  # readIndex.addRequest
                    if len(self.pending_reads) == RQ:  # the queue is full: dropped, no heartbeat
                        self.drops += 1
                        return
                    self.pending_reads.append([m["hint"], self.committed, {self.s}, f])
                for i in range(self.sim.R):
                    if i != self.s and i in self.members:
                        self.send(msg(HEARTBEAT, i + 1, commit=min(self.remotes[i].match, self.committed),
                                      hint=m["hint"]))
        elif self.role == FOLLOWER and self.leader != 0 and f == self.s:
            fw = dict(m)
            fw.update(to=self.leader, term=0)
            self.send(fw)
        else:
            self.drops += 1

    # -- follower --
    def on_replicate(self, m):
        resp = msg(REPLICATE_RESP, m["frm"])
        if m["log_index"] < self.committed:
            resp["log_index"] = self.committed
            self.send(resp)
            return
        n = m["nent"]
        if self.term_at(m["log_index"]) == m["log_term"]:
            conflict = None
            for k, e in enumerate(m["ents"]):
                if self.term_at(m["log_index"] + 1 + k) != e.term:
                    conflict = k
                    break
            last_new = m["log_index"] + n
            if conflict is not None:
                ci = m["log_index"] + 1 + conflict
                if ci > self.committed and (last_new > self.cap_base + self.sim.cfg["log_capacity"] or
                                            not self.stream_fits(sum(e.chunks for e in m["ents"][conflict:]))):
                    self.drops += 1
                    return
                if ci <= self.committed:
                    self.err |= ERR_CONFLICT
                else:
                    del self.log[ci - self.marker - 1:]
                    for e in m["ents"][conflict:]:
                        ne = Entry(e.term, e.type, e.data, e.cc)
                        if ne.crc != e.crc:
                            self.err |= ERR_CRC
                        self.put(ne)
            self.commit_to(min(last_new, m["commit"]))
            resp["log_index"] = last_new
        else:
            resp.update(reject=1, log_index=m["log_index"], hint=self.last)
        self.send(resp)

    def on_install_snapshot(self, m):
        resp = msg(REPLICATE_RESP, m["frm"])
        si, st = m["log_index"], m["log_term"]
        if si <= self.committed:
            resp["log_index"] = self.committed
        elif self.term_at(si) == st:
            self.commit_to(si)
            resp["log_index"] = self.committed
        else:
            self.log = []
            self.marker = self.committed = self.snap_index = self.processed = si
            self.marker_term = self.snap_term = st
            self.applied = max(self.applied, si)
            self.members = {k for k in range(8) if m["hint_high"] >> k & 1}  # the snapshot's membership
            self.snap_members = set(self.members)
            self.restored_at = si
            resp["log_index"] = self.last
        self.send(resp)

    # -- elections --
    def campaign(self):
        self.become_candidate()
        self.votes[self.s] = True
        if sum(1 for k, v in self.votes.items() if v and k in self.members) == self.quorum:
            self.become_leader()
            return
        for i in range(self.sim.R):
            if i != self.s and i in self.members:
                self.send(msg(REQUEST_VOTE, i + 1, term=self.term, log_index=self.last,
                              log_term=self.term_at(self.last)))

    def on_request_vote(self, m):
        grant = self.vote in (0, m["frm"]) and self.up_to_date(m["log_index"], m["log_term"])
        if grant:
            self.etick = 0
            self.vote = m["frm"]
        self.send(msg(REQUEST_VOTE_RESP, m["frm"], reject=0 if grant else 1))

    def on_vote_resp(self, m):
        f = m["frm"] - 1
        if f not in self.votes:
            self.votes[f] = not m["reject"]
        yes = sum(1 for k, v in self.votes.items() if v and k in self.members)
        total = sum(1 for k in self.votes if k in self.members)
        if yes == self.quorum:
            self.become_leader()
            self.broadcast_replicate()
        elif total - yes == self.quorum:
            self.become_follower(self.term, 0)

    # -- Handle --
    def local(self, t):
        self.handle(msg(t, self.id, frm=self.id))

    def tick(self):
        c = self.sim.cfg
        if self.role == LEADER:
            self.etick += 1
            if self.etick >= c["election_rtt"]:
                self.etick = 0
                if c["check_quorum"]:
                    self.local(CHECK_QUORUM)
            self.htick += 1
            if self.htick >= c["heartbeat_rtt"]:
                self.htick = 0
                self.local(LEADER_HEARTBEAT)
        else:
            self.etick += 1
            if self.s in self.members and self.etick >= self.rand_to:  # selfRemoved: no elections
                self.etick = 0
                self.local(ELECTION)

    def handle(self, m):
        c = self.sim.cfg
        t, mt = m["type"], m["term"]
        if mt != 0 and mt != self.term:
            if (t == REQUEST_VOTE and c["check_quorum"] and mt > self.term and m["hint"] != m["frm"]
                    and self.leader != 0 and self.etick < c["election_rtt"]):
                return
            if mt > self.term:
                self.become_follower(mt, m["frm"] if t in LEADER_MSGS else 0)
            else:
                if c["check_quorum"] and t in LEADER_MSGS:
                    self.send(msg(NOOP, m["frm"]))
                return
        role = self.role
        if t == LOCAL_TICK:
            self.tick()
        elif t == ELECTION:
            if role != LEADER and self.s in self.members and not self.committed > self.applied:
                if self.term >= TERM_MAX:
                    self.err |= ERR_TERM
                else:
                    self.campaign()
        elif t == LEADER_HEARTBEAT:
            if role == LEADER:  # a pending ReadIndex rides on every heartbeat (readIndex.peepCtx)
                ctx = self.pending_reads[-1][0] if self.pending_reads else 0
                for i in range(self.sim.R):
                    if i != self.s and i in self.members:
                        self.send(msg(HEARTBEAT, i + 1, commit=min(self.remotes[i].match, self.committed), hint=ctx))
        elif t == CHECK_QUORUM:
            if role == LEADER:
                c_act = len((self.active | {self.s}) & self.members)
                self.active = set()
                if c_act < self.quorum:
                    self.become_follower(self.term, 0)
        elif t == PROPOSE:  # the message carries its Cmds (m["ents"]), or a membership change
            cc = m["hint_high"]
            if role == LEADER:
                dropped = bool(cc) and self.cc_pending  # one change at a time: an empty entry instead
                if not self.append(m["nent"], [] if cc else [e.data for e in m["ents"]], 0 if dropped else cc):
                    self.drops += 1
                    return
                if dropped:
                    self.drops += 1
                elif cc:
                    self.cc_pending = True
                self.broadcast_replicate()
            elif role == FOLLOWER and self.leader != 0 and m["src_b"] == 0:
                f = dict(m)
                f.update(to=self.leader, term=0, src_b=m["src_b"] + 1)
                self.send(f)
            else:
                self.drops += 1
        elif t in (REPLICATE, HEARTBEAT, INSTALL_SNAPSHOT):
            if role == LEADER:
                return
            if role == CANDIDATE:
                self.become_follower(self.term, m["frm"])
            else:
                self.etick = 0
                self.leader = m["frm"]
            if t == REPLICATE:
                self.on_replicate(m)
            elif t == HEARTBEAT:
                self.commit_to(m["commit"])
                self.send(msg(HEARTBEAT_RESP, m["frm"], hint=m["hint"], hint_high=m["hint_high"]))
            else:
                self.on_install_snapshot(m)
        elif t == REPLICATE_RESP:
            if role == LEADER:
                self.on_replicate_resp(m)
        elif t == HEARTBEAT_RESP:
            if role == LEADER:
                self.on_heartbeat_resp(m)
        elif t == READ_INDEX:
            self.on_read_index(m)
        elif t == READ_INDEX_RESP:
            if role == FOLLOWER:
                self.etick = 0
                self.leader = m["frm"]
                self.read_ready_add(m["hint"], m["log_index"])
        elif t == REQUEST_VOTE:
            self.on_request_vote(m)
        elif t == REQUEST_VOTE_RESP:
            if role == CANDIDATE:
                self.on_vote_resp(m)

    # -- membership: raft.addNode / removeNode through the rsm's ApplyConfigChange --
    def apply_config_change(self, cc):
        op, slot = cc >> 4, (cc & 0xF) - 1
        self.cc_pending = False
        if slot >= self.sim.R:
            return
        if op == CC_ADD:
            if slot in self.members:
                return
            self.members.add(slot)
            self.remotes[slot] = Remote(0, self.last + 1)
        elif op == CC_REMOVE:
            self.members.discard(slot)
            self.active.discard(slot)
            if slot == self.s and self.role == LEADER:
                self.become_follower(self.term, 0)
            if self.role == LEADER and self.members and self.try_commit():
                self.broadcast_replicate()

    # -- views (same field names as the C views) --
    def view(self):
        R = self.sim.R
        return dict(
            term=self.term, vote=self.vote, leader=self.leader, committed=self.committed,
            applied=self.applied, last=self.last, marker=self.marker, marker_term=self.marker_term,
            snap_index=self.snap_index, snap_term=self.snap_term, cap_base=self.cap_base, processed=self.processed,
            role=self.role, election_tick=self.etick, heartbeat_tick=self.htick,
            rand_timeout=self.rand_to, rng_ctr=self.rng,
            granted=sum(1 << k for k, v in self.votes.items() if v),
            responded=sum(1 << k for k in self.votes),
            active=sum(1 << k for k in self.active), err=self.err, drops=self.drops & 0xFFFFFFFF,
            members=sum(1 << k for k in self.members), snap_members=sum(1 << k for k in self.snap_members),
            cc_pending=int(self.cc_pending),
            match=[r.match for r in self.remotes][:R], next=[r.next for r in self.remotes][:R],
            rsnap=[r.snap for r in self.remotes][:R], rstate=[r.state for r in self.remotes][:R],
        )


class Sim:
    """All replicas of all groups, one process, in-memory router."""

    def __init__(self, **cfg):
        from .pyoracle import default_config  # same defaults; no code shared with oracle.c
        self.cfg = default_config(**cfg)
        self.G, self.R = self.cfg["groups"], self.cfg["replicas"]
        P, L = self.cfg["payload_bytes"], self.cfg["log_capacity"]
        self.maxc = self.cfg.get("max_cmd_bytes", 0) or P
        full = (L * ((P + 15) // 16 * 16) + 4095) // 4096
        big = 2 * ((self.maxc + 4095) // 4096 + 1) if self.maxc > P else 0  # room for two of the longest Cmds
        pts = 16
        while pts < 2 * full + big:
            pts <<= 1
        self.pts = (self.cfg.get("stream_pages", 0) or pts) if P else 1
        self.t = 0
        self.isolate = None
        self.reps = [Replica(self, g, s) for g in range(self.G) for s in range(self.R)]
        self._pay = {}
        self.staged = {}  # window group -> (slot, [cmd bytes]) for the next tick (propose)
        self.reads = {}   # window rid -> ReadIndex ctx for the next tick
        self.ccs = {}     # window group -> (slot, descriptor) membership change for the next tick

    def compact(self, group, index):
        """rg_compact between ticks: every replica of `group` compacts to min(index, snap_index) when
        that is above its marker; the next step releases the stream below (fidx)."""
        base = self.cfg["group_base"]
        if not (base <= group < base + self.G):
            return -1
        n = 0
        for s in range(self.R):
            r = self.reps[(group - base) * self.R + s]
            c = min(index, r.snap_index)
            if c <= r.marker:
                continue
            mt = r.term_at(c)
            del r.log[:c - r.marker]
            r.marker, r.marker_term = c, mt
            r.fidx = c + 1
            n += 1
        return n

    def config_change(self, group, slot, op, target):
        base = self.cfg["group_base"]
        if not (base <= group < base + self.G) or slot >= self.R or target >= self.R or op not in (CC_ADD, CC_REMOVE):
            return -1
        if group - base in self.ccs:
            return -3
        self.ccs[group - base] = (slot, op << 4 | (target + 1))
        return 0

    def read_index(self, reqs):
        base = self.cfg["group_base"]
        for g, s, ctx in reqs:
            if not (base <= g < base + self.G) or s >= self.R or ctx == 0:
                return -1
        for g, s, ctx in reqs:
            self.reads[(g - base) * self.R + s] = ctx
        return 0

    def read_ready(self, rid):
        rr = self.reps[rid].ready_reads
        return list(rr[1]) if rr is not None and rr[0] == self.t - 1 else []

    def propose(self, batches):
        """Stage caller proposals (group, slot, [cmds]) for the next tick; all or nothing:
        0, -1 (invalid) or -3 (a group's batch is full / has a second slot)."""
        c = self.cfg
        E, P, base = c["max_entries_per_msg"], c["payload_bytes"], c["group_base"]
        new = {g: (s, list(v)) for g, (s, v) in self.staged.items()}
        for g, s, cmds in batches:
            if not (base <= g < base + self.G) or s >= self.R or not 1 <= len(cmds) <= E:
                return -1
            if any(len(x) > self.maxc for x in cmds):
                return -1
            lg = g - base
            if lg in new and new[lg][1] and new[lg][0] != s:
                return -3
            cur = new.setdefault(lg, (s, []))[1]
            if len(cur) + len(cmds) > E:
                return -3
            cur.extend(bytes(x) for x in cmds)
        self.staged = new
        return 0

    def payload(self, slab, g, k):
        key = (slab, g, k)
        if key not in self._pay:
            self._pay[key] = payload(self.cfg["seed"], slab, g, k, self.cfg["payload_bytes"])
        return self._pay[key]

    def lost(self, rep, dst, n):
        rid = rep.g * self.R + rep.s
        if self.isolate is not None and (self.isolate[rid] or self.isolate[rep.g * self.R + dst]):
            return True
        ppm = self.cfg["drop_ppm"]
        if ppm:
            h = mix64(self.cfg["seed"] ^ mix64((self.t << 40) ^ (rid << 8) ^ dst) ^ (n + 1))
            return h % 1000000 < ppm
        return False

    def bootstrap(self):
        """A joining slot (join_slots) starts empty at term 0 with no membership; the others with one
        ConfigChange entry per slot at term 1: AddNode(s) for each initial member, 0 for the rest."""
        R = self.R
        js = self.cfg.get("join_slots", 0)
        im = (self.cfg.get("initial_members", 0) or (1 << R) - 1) & ~js
        for r in self.reps:
            joining = js >> r.s & 1
            r.rng = 0
            r.hw = r.lpg = r.nlpg = r.fidx = 0
            r.members = set() if joining else {k for k in range(R) if im >> k & 1}
            r.snap_members = set(r.members)
            r.log = []
            r.become_follower(0 if joining else 1, 0)
            last = 0 if joining else R
            r.log = [Entry(1, 1, b"", (CC_ADD << 4 | (k + 1)) if im >> k & 1 else 0) for k in range(last)]
            r.committed = last
            r.remotes = [Remote(0, last + 1) for _ in range(R)]
            r.out, r.emitted = {}, {}
        self.t = 0

    def tick(self, prop_target=None, prop_count=None, campaign=None, isolate=None, flags=0):
        if prop_target is not None and self.staged:
            raise ValueError("tick-input proposals while caller proposals are staged")
        staged, self.staged = self.staged, {}
        reads, self.reads = self.reads, {}
        ccs, self.ccs = self.ccs, {}
        self.isolate = isolate
        inbox = {id(r): [] for r in self.reps}
        for r in self.reps:  # deliver last tick's outboxes
            for d, lst in r.out.items():
                dst = self.reps[r.g * self.R + d]
                inbox[id(dst)].append((r.s, lst))
        for r in self.reps:
            r._inbox = sorted(inbox[id(r)], key=lambda x: x[0])
        for r in self.reps:
            r.out, r.emitted = {}, {}
        for g in range(self.G):
            for s in range(self.R):
                r = self.reps[g * self.R + s]
                marker_start, processed_start = r.marker, r.processed
                r.restored_at = 0
                r.nlpg = r.lpg  # the pages below the last step's compaction go back when this step ends
                if r.fidx:
                    r.nlpg = (r.log[r.fidx - r.marker - 1].pos if r.fidx <= r.last else r.hw) >> 8
                for _, lst in r._inbox:
                    for m in lst:
                        r.handle(m)
                rid = g * self.R + s
                if campaign is not None and campaign[rid]:
                    r.local(ELECTION)
                if not flags & 1:
                    r.local(LOCAL_TICK)
                slab = self.t % self.cfg["num_slabs"]
                cmds = None
                if prop_target is not None and prop_target[g] == s and prop_count[g] > 0:
                    P = self.cfg["payload_bytes"]
                    cmds = [self.payload(slab, g, k) if P else b"" for k in range(int(prop_count[g]))]
                elif g in staged and staged[g][0] == s:
                    cmds = staged[g][1]
                if cmds:
                    hm = sum(1 << k for k, x in enumerate(cmds) if x)
                    r.handle(msg(PROPOSE, r.id, frm=r.id, nent=len(cmds), hint=hm, src_a=slab, src_b=0,
                                 ents=tuple(Entry(0, 0, x) for x in cmds)))
                if g in ccs and ccs[g][0] == s:
                    r.handle(msg(PROPOSE, r.id, frm=r.id, nent=1, hint=0, hint_high=ccs[g][1], src_a=slab,
                                 src_b=0, ents=()))
                if reads.get(rid):
                    r.handle(msg(READ_INDEX, r.id, frm=r.id, hint=reads[rid]))
                i = max(processed_start, r.restored_at) + 1
                while i <= r.committed:  # a removal may commit more: those are handed over too
                    e = r.log[i - r.marker - 1]
                    if e.type == 1 and e.cc:
                        r.apply_config_change(e.cc)
                    i += 1
                r.processed = r.committed  # handed to the state machine this step
                if not self.cfg["apply_feedback"]:
                    r.applied = r.processed
                se, co = self.cfg["snapshot_entries"], self.cfg["compaction_overhead"]
                if se and r.applied >= r.snap_index and r.applied - r.snap_index >= se:
                    r.snap_index, r.snap_term = r.applied, r.term_at(r.applied)
                    r.snap_members = set(r.members)
                    cpt = r.snap_index - co if r.snap_index > co else 0
                    if cpt > r.marker:
                        mt = r.term_at(cpt)
                        del r.log[:cpt - r.marker]
                        r.marker, r.marker_term = cpt, mt
                r.cap_base = marker_start
                r.lpg = r.nlpg
                r.fidx = r.marker + 1 if r.marker != marker_start else 0
        self.t += 1

    # views
    def replica(self, rid):
        return self.reps[rid].view()

    def msgs(self, rid, dst):
        out = []
        for m in self.reps[rid].out.get(dst, []):
            d = {k: m[k] for k in ("type", "to", "reject", "nent", "term", "log_term", "log_index",
                                   "commit", "hint", "hint_high", "src_a", "src_b")}
            d["from"] = m["frm"]
            d["terms"] = [e.term for e in m["ents"]] if m["type"] == REPLICATE else []
            out.append(d)
        return out

    def entry(self, rid, index):
        r = self.reps[rid]
        if not (r.marker < index <= r.last):
            return None
        e = r.log[index - r.marker - 1]
        return dict(term=e.term, type=e.type, len=e.len, crc=e.crc)

    # -- scenario helpers (KATs): same contract as or_import_replica / or_deliver --
    def import_replica(self, rid, view: dict, terms, types=None, payloads=None, lens=None):
        r = self.reps[rid]
        P = self.cfg["payload_bytes"]
        at = 0  # the Cmds come packed back to back (application entries with a Cmd)
        for k in ("term", "vote", "leader", "committed", "applied", "processed", "marker", "marker_term",
                  "snap_index", "snap_term", "cap_base", "role", "err", "drops"):
            setattr(r, k, view.get(k, 0))
        r.etick = view.get("election_tick", 0)
        r.htick = view.get("heartbeat_tick", 0)
        r.rand_to = view.get("rand_timeout", 0)
        r.rng = view.get("rng_ctr", 0)
        g = view.get("granted", 0)
        resp = view.get("responded", 0)
        r.votes = {k: bool(g >> k & 1) for k in range(8) if resp >> k & 1}
        r.active = {k for k in range(8) if view.get("active", 0) >> k & 1}
        r.pending_reads, r.ready_reads = [], None
        r.members = {k for k in range(8) if view.get("members", (1 << self.R) - 1) >> k & 1}
        r.snap_members = {k for k in range(8) if view.get("snap_members", view.get("members", (1 << self.R) - 1)) >> k & 1}
        r.cc_pending = bool(view.get("cc_pending", 0))
        r.log = []
        r.hw = r.lpg = r.nlpg = r.fidx = 0  # a fresh payload stream (rg_import_replica)
        for k, t in enumerate(terms):
            ty = 0 if types is None else types[k] & 0xFF
            ln = P if lens is None else lens[k]
            empty = types is not None and types[k] & 0x100
            data = b""
            if payloads is not None and P and ty == 0 and not empty:
                data = payloads[at:at + ln]
                at += ln
            r.put(Entry(t, ty, bytes(data), ln if ty == 1 and lens is not None else 0))
        assert r.last == view.get("last", r.last)
        r.remotes = []
        for k in range(self.R):
            rp = Remote(view.get("match", [0] * 8)[k], view.get("next", [0] * 8)[k])
            rp.snap = view.get("rsnap", [0] * 8)[k]
            rp.state = view.get("rstate", [0] * 8)[k]
            r.remotes.append(rp)

    def notify_applied(self, rid, index):
        """Peer.NotifyRaftLastApplied (index <= processed)."""
        r = self.reps[rid]
        if index > r.processed:
            return -1
        r.applied = index
        return 0

    def deliver(self, rid_src, **f):
        r = self.reps[rid_src]
        m = msg(f.get("type"), f.get("to"))
        for k, v in f.items():
            m["frm" if k == "from" else k] = v
        if "from" not in f:
            m["frm"] = r.id
        if m["type"] == REPLICATE and m["nent"]:
            lo = m["log_index"] + 1
            m["ents"] = tuple(r.log[lo - r.marker - 1: lo - r.marker - 1 + m["nent"]])
        r.out.setdefault(m["to"] - 1, []).append(m)
