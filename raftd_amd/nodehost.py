"""The NodeHost subset raftd calls, re-implemented over the step engine.

raftd reaches Raft only through dragonboat's NodeHost (`/root/reference/raft/raft_manager.go:109,
142-144,159,173,184`, `raft/members.go:21,30`). The production binding is a cgo package
(`INTEGRATION.md`); no Go toolchain exists here, so this module is the same shim in Python, over
`raftd_amd.engine.Engine`, with dragonboat's method names, argument meaning and error behaviour:

    NodeHost.StartOnDiskReplica(initialMembers, join, create, config)   raft_manager.go:142-144
    NodeHost.SyncRequestAddReplica(shardID, replicaID, target, cci)     raft_manager.go:173
    NodeHost.SyncRequestDeleteReplica(shardID, replicaID, cci)          raft_manager.go:184
    NodeHost.GetLeaderID(shardID) -> (leaderID, term, valid)             members.go:21
    NodeHost.SyncGetShardMembership(shardID) -> Membership              members.go:30
    NodeHost.Close()                                                     raft_manager.go:159

Replica identity. raftd names replicas by arbitrary uint64 IDs (`env.ReplicaID`, RecruitReplica's
`replicaID`); the engine names them by slot, 0 .. R-1 of each shard, fixed at `rg_create`. The shim
keeps the map a cgo shim must keep, per shard:
- `StartOnDiskReplica`'s initial members take slots 0 .. k-1 in ascending replica-ID order (the
  engine's `initial_members`); slots k .. R-1 are provisioned as join slots (`join_slots`: empty log,
  term 0, outside the membership — a node started with `join = true`).
- `SyncRequestAddReplica` gives a new replica ID the lowest free slot. A slot that held a removed
  replica is first reset to a fresh joiner (`import_replica` of the join state), so the new replica
  starts with an empty log, as a new dragonboat node does. The ConfigChange is proposed at the
  leader's slot; the call ticks the shard until the leader has applied it (dragonboat's Sync*
  semantics) or the deadline passes (`ErrTimeout`).
- A removed replica ID can never be added again (dragonboat: `ErrReplicaRemoved`); more replicas
  than slots at once is `ErrRejected` (this engine's bound: R <= 8 per shard).

The shim drives ticks itself (`tick()`, dragonboat's tick goroutine at `RTTMillisecond`); a Sync*
call ticks until its change is applied. Deadlines are counted in ticks (raftd's 10 s at 3 ms RTT =
3,333 ticks).

Two shims share this vocabulary:
- `NodeHost` — ONE node: raftd runs one NodeHost per process (`raft_manager.go:102-109`), and here a
  node is one rank of the spread placement (every replica of a shard on its own rank,
  emulating separate machines). The node hosts one replica of each shard, decides `join` for itself
  (`raft_manager.go:134-144`), answers GetLeaderID and SyncGetShardMembership from its own replica
  (`members.go:20-50`), and completes a membership request when its own replica has applied it.
- `ColocatedNodeHost` — every replica of a shard in one engine (one process hosting all the
  shard's nodes): r03's shim, kept for single-GPU deployments and tests.
"""
from __future__ import annotations

from dataclasses import dataclass, field

CC_ADD, CC_REMOVE = 1, 2  # rg_config_change ops (include/raftgpu.h RG_CC_*)
LEADER = 2


class NodeHostError(Exception):
    """dragonboat's request errors, by name."""


class ErrShardNotFound(NodeHostError):
    pass


class ErrTimeout(NodeHostError):
    pass


class ErrRejected(NodeHostError):
    pass


class ErrReplicaRemoved(NodeHostError):
    pass


class ErrInvalidOperation(NodeHostError):
    pass


@dataclass
class Membership:
    """dragonboat's Membership: Nodes = voting members {replicaID: address}; Removed = IDs removed."""
    nodes: dict = field(default_factory=dict)
    removed: set = field(default_factory=set)


@dataclass
class _Shard:
    ids: list          # slot -> replica ID (0 = free)
    addrs: list        # slot -> address
    removed: set = field(default_factory=set)
    stale: set = field(default_factory=set)  # slots whose replica was removed (reset before reuse)


def join_view(R: int) -> dict:
    """The replica state of a node started with join = true: term 0, empty log,
    outside the membership."""
    return dict(term=0, vote=0, leader=0, committed=0, applied=0, last=0, marker=0, marker_term=0,
                snap_index=0, snap_term=0, cap_base=0, processed=0, role=0, election_tick=0, heartbeat_tick=0,
                rand_timeout=10, rng_ctr=1, granted=0, responded=0, active=0, err=0, drops=0, members=0,
                snap_members=0, cc_pending=0, match=[0] * 8, next=[1] * 8, rsnap=[0] * 8, rstate=[0] * 8)



def bootstrap_view(group: int, slot: int, members: int, replicas: int, cfg: dict) -> tuple:
    """(view, terms, types, lens) of a replica started by StartOnDiskReplica(initialMembers, join=false)
    whose shard's initial membership is the slot mask `members` (becomeFollower(1), one
    ConfigChange entry per slot at term 1 — AddNode for the members, descriptor 0 for the others —
    committed), as rg_bootstrap builds it with rg_config.initial_members = members."""
    from .wal import mix64
    R, ET = replicas, cfg["election_rtt"]
    key = (group << 32) | (slot << 24) | 1
    rto = ET + mix64(cfg["seed"] ^ mix64(key)) % ET
    view = dict(term=1, vote=0, leader=0, committed=R, applied=0, last=R, marker=0, marker_term=0,
                snap_index=0, snap_term=0, cap_base=0, processed=0, role=0, election_tick=0, heartbeat_tick=0,
                rand_timeout=rto, rng_ctr=1, granted=0, responded=0, active=0, err=0, drops=0, members=members,
                snap_members=members, cc_pending=0, match=[0] * 8, next=[R + 1] * 8, rsnap=[0] * 8,
                rstate=[0] * 8)
    lens = [(CC_ADD << 4 | (k + 1)) if (members >> k) & 1 else 0 for k in range(R)]
    return view, [1] * R, [1] * R, lens


@dataclass
class RequestState:
    """dragonboat's RequestState of a membership request: `done` once the node's own replica has
    applied the change, `error` an ErrTimeout / ErrRejected instance, or None."""
    shard: int
    op: int
    slot: int
    replica_id: int
    deadline: int
    done: bool = False
    error: Exception | None = None
    proposed_at: int = -1


class NodeHost:
    """dragonboat.NodeHost's subset for ONE node (one rank of the spread placement).

    host: the node's engine share, addressed by (global shard, slot) — raftd_amd.cluster.DistEngine
    (one rank per process) or RankView (a rank of a whole-cluster backend, tests). It provides
    hosts(shard, slot), replica_of, import_replica_of, config_change, tick and t.
    directory: the deployment's node table by rank, [(replicaID, raftAddress)] — raftd's env.ReplicaID
    / RAFT_LISTEN_ADDR of the node on each rank (a cgo shim gets it from its launcher). Slot s of shard
    g is replica directory[rank_of(g, s)]: the node hosting it. Requires ranks >= replicas (one
    replica of a shard per node).

    tick model: step() = before_tick() + host.tick() + after_tick(). When several NodeHosts share one
    backend (RankView), the driver calls before_tick() on each, ticks the backend once, then
    after_tick() on each. Sync* requests tick through step() until the node's own replica applied the
    change: use them when this NodeHost drives the ticks; with several ranks ticking in lockstep, use
    the Request* calls and poll their RequestState."""

    def __init__(self, host, replicas: int, directory, nhc: dict | None = None, retry_ticks: int = 20):
        from .cluster import rank_of
        self.h, self.R = host, replicas
        self.N, self.rank = host.N, host.rank
        self.dir = [(int(i), str(a)) for i, a in directory]
        if len(self.dir) != self.N:
            raise ErrInvalidOperation(f"a directory of {len(self.dir)} nodes for {self.N} ranks")
        if self.N < replicas:
            raise ErrInvalidOperation(f"{self.N} nodes for {replicas} replica slots: a node would host two "
                                      "replicas of one shard (use ColocatedNodeHost)")
        if len({i for i, _ in self.dir}) != self.N or any(i == 0 for i, _ in self.dir):
            raise ErrInvalidOperation("node replica IDs must be distinct and non-zero")
        self.replica_id, self.address = self.dir[self.rank]
        self.rank_of = rank_of
        self.nhc = dict(nhc or {})
        self.retry = retry_ticks
        self.shards: dict[int, int] = {}  # shard -> the local slot
        self.removed: dict[int, set] = {}
        self.pending: list[RequestState] = []
        self.staged: list = []            # (shard, slot, op, target) staged for the next tick (tests)
        self.closed = False

    # ---- identity
    def slot_of(self, shard: int, replica_id: int) -> int:
        """The slot of shard `shard` hosted by node `replica_id` (-1: that node hosts none)."""
        for s in range(self.R):
            if self.dir[self.rank_of(shard, s, self.N)][0] == replica_id:
                return s
        return -1

    def id_of(self, shard: int, slot: int) -> int:
        return self.dir[self.rank_of(shard, slot, self.N)][0]

    def _check_open(self):
        if self.closed:
            raise ErrInvalidOperation("NodeHost closed")

    def _local(self, shard_id: int) -> int:
        self._check_open()
        s = self.shards.get(shard_id)
        if s is None:
            raise ErrShardNotFound(f"shard {shard_id} not started on node {self.replica_id}")
        return s

    def _view(self, shard_id: int) -> dict:
        return self.h.replica_of(shard_id, self._local(shard_id))

    # ---- raft_manager.go:142-144
    def StartOnDiskReplica(self, initial_members: dict | None, join: bool, create=None, config: dict | None = None):
        """Start this node's replica of shard config['ShardID'] — as a bootstrapping member of
        `initial_members` {replicaID: addr} (join = false), or as a joining replica (join = true,
        initial_members None) that becomes a member when the shard's leader recruits it. raftd decides
        join per node from RAFT_INITIAL_MEMBERS (raft_manager.go:134-139). Every node of the shard
        starts its replica before the first tick."""
        self._check_open()
        config = dict(config or {})
        sid = int(config.get("ShardID", 0))
        if sid in self.shards:
            raise ErrInvalidOperation(f"shard {sid} already started on node {self.replica_id}")
        if self.h.t != 0:
            raise ErrInvalidOperation("StartOnDiskReplica after the engine started ticking")
        s = self.slot_of(sid, self.replica_id)
        if s < 0:
            raise ErrInvalidOperation(f"node {self.replica_id} hosts no replica of shard {sid}")
        if join:
            if initial_members:
                raise ErrInvalidOperation("join = true with initial members")
            self.h.import_replica_of(sid, s, join_view(self.R), [], [], b"")
        else:
            ids = {int(i) for i in (initial_members or {})}
            if self.replica_id not in ids:
                raise ErrInvalidOperation(f"node {self.replica_id} is not one of the initial members {sorted(ids)}")
            unknown = ids - {i for i, _ in self.dir}
            if unknown:
                raise ErrInvalidOperation(f"initial members {sorted(unknown)} are not nodes of this deployment")
            mask = sum(1 << k for k in range(self.R) if self.id_of(sid, k) in ids)
            cfg = getattr(self.h, "cfg", None) or self.h.b.cfg
            view, terms, types, lens = bootstrap_view(sid, s, mask, self.R, cfg)
            self.h.import_replica_of(sid, s, view, terms, types, None, lens)
        self.shards[sid] = s
        self.removed[sid] = set()
        if create is not None:
            create(sid, self.replica_id)

    # ---- ticking (dragonboat's tick goroutine)
    def before_tick(self):
        """Stage this node's membership proposals for the next tick: a request not yet applied is
        proposed at the node's own replica (a follower forwards it to its leader), and proposed again
        every retry_ticks ticks while it is not applied (a proposal can be dropped: no leader known,
        a change already in flight, a lost forward)."""
        self._check_open()
        self.staged = []
        t = self.h.t
        busy = set()
        for rq in self.pending:
            if rq.done or rq.error or rq.shard in busy:
                continue
            if rq.proposed_at < 0 or t - rq.proposed_at >= self.retry:
                s = self.shards[rq.shard]
                self.h.config_change(rq.shard, s, rq.op, rq.slot)  # one change per shard per tick
                self.staged.append((rq.shard, s, rq.op, rq.slot))
                rq.proposed_at = t
                busy.add(rq.shard)

    def after_tick(self):
        """Complete the requests the node's own replica has applied; time out the others."""
        t = self.h.t
        for rq in self.pending:
            if rq.done or rq.error:
                continue
            members = self._view(rq.shard)["members"]
            has = bool((members >> rq.slot) & 1)
            if has == (rq.op == CC_ADD):
                rq.done = True
                if rq.op == CC_REMOVE:
                    self.removed[rq.shard].add(rq.replica_id)
            elif t >= rq.deadline:
                rq.error = ErrTimeout(f"shard {rq.shard}: membership change op {rq.op} of replica "
                                      f"{rq.replica_id} not applied by tick {rq.deadline}")
        self.pending = [rq for rq in self.pending if not (rq.done or rq.error)]

    def step(self, **inputs):
        """One tick of this node: before_tick, the engine's tick (collective across ranks), after_tick."""
        self.before_tick()
        self.h.tick(**inputs)
        self.after_tick()

    def _request(self, shard_id: int, op: int, replica_id: int, deadline_ticks: int) -> RequestState:
        self._local(shard_id)
        if replica_id == 0:
            raise ErrInvalidOperation("replica ID 0")
        if op == CC_ADD and replica_id in self.removed[shard_id]:
            raise ErrReplicaRemoved(f"replica {replica_id} was removed from shard {shard_id}")
        slot = self.slot_of(shard_id, replica_id)
        if slot < 0:
            raise ErrRejected(f"node {replica_id} hosts no replica slot of shard {shard_id}")
        rq = RequestState(shard_id, op, slot, replica_id, self.h.t + deadline_ticks)
        if bool((self._view(shard_id)["members"] >> slot) & 1) == (op == CC_ADD):
            rq.done = True  # already a member / already removed
            return rq
        self.pending.append(rq)
        return rq

    # ---- raft_manager.go:165-174 (RecruitReplica) / :176-185 (RemoveReplica), asynchronous forms
    def RequestAddReplica(self, shard_id: int, replica_id: int, target: str, config_change_index: int = 0,
                          deadline_ticks: int = 3333) -> RequestState:
        known = dict(self.dir)
        if replica_id in known and known[replica_id] != target:
            raise ErrRejected(f"node {replica_id} listens on {known[replica_id]}, not {target}")
        return self._request(shard_id, CC_ADD, replica_id, deadline_ticks)

    def RequestDeleteReplica(self, shard_id: int, replica_id: int, config_change_index: int = 0,
                             deadline_ticks: int = 3333) -> RequestState:
        return self._request(shard_id, CC_REMOVE, replica_id, deadline_ticks)

    def _sync(self, rq: RequestState):
        while not (rq.done or rq.error):
            self.step()
        if rq.error:
            raise rq.error

    def SyncRequestAddReplica(self, shard_id: int, replica_id: int, target: str, config_change_index: int = 0,
                              deadline_ticks: int = 3333):
        self._sync(self.RequestAddReplica(shard_id, replica_id, target, config_change_index, deadline_ticks))

    def SyncRequestDeleteReplica(self, shard_id: int, replica_id: int, config_change_index: int = 0,
                                 deadline_ticks: int = 3333):
        self._sync(self.RequestDeleteReplica(shard_id, replica_id, config_change_index, deadline_ticks))

    # ---- members.go:21 — the leader as this node's replica knows it
    def GetLeaderID(self, shard_id: int):
        """(leader replica ID, term, valid) from this node's own replica of the shard."""
        v = self._view(shard_id)
        if v["leader"] == 0:
            return 0, v["term"], False
        return self.id_of(shard_id, v["leader"] - 1), v["term"], True

    # ---- members.go:30 — the membership this node's replica has applied
    def SyncGetShardMembership(self, shard_id: int) -> Membership:
        v = self._view(shard_id)
        addr = dict(self.dir)
        nodes = {}
        for s in range(self.R):
            if (v["members"] >> s) & 1:
                i = self.id_of(shard_id, s)
                nodes[i] = addr[i]
        return Membership(nodes=nodes, removed=set(self.removed[shard_id]))

    # ---- raft_manager.go:159
    def Close(self):
        self.closed = True


class ColocatedNodeHost:
    """dragonboat.NodeHost's subset over one engine that hosts EVERY replica of its shards (the
    co-located layout: all of a shard's nodes in one process, e.g. a single-GPU deployment or a test).
    `engine` is a raftd_amd.engine.Engine (or any object with its tick / config_change / leader /
    replica / import_replica methods). For one NodeHost per node (replicas on different ranks), see
    NodeHost."""

    def __init__(self, engine, replicas: int, nhc: dict | None = None):
        self.e = engine
        self.R = replicas
        self.nhc = dict(nhc or {})  # WALDir, NodeHostDir, RTTMillisecond, RaftAddress (raft_manager.go:101-106)
        self.shards: dict[int, _Shard] = {}
        self.closed = False

    # ---- the engine config a NodeHost needs for StartOnDiskReplica's initial membership
    @staticmethod
    def engine_slots(initial_members: dict, replicas: int) -> dict:
        """rg_config fields for `initial_members` {replicaID: addr}: the initial members take slots
        0..k-1 (ascending ID) and the other slots start as join slots."""
        k = len(initial_members)
        if not 1 <= k <= replicas:
            raise ErrInvalidOperation(f"{k} initial members for {replicas} replica slots")
        im = (1 << k) - 1
        return dict(initial_members=im, join_slots=((1 << replicas) - 1) & ~im)

    def _check_open(self):
        if self.closed:
            raise ErrInvalidOperation("NodeHost closed")

    def _shard(self, shard_id: int) -> _Shard:
        self._check_open()
        s = self.shards.get(shard_id)
        if s is None:
            raise ErrShardNotFound(f"shard {shard_id} not found")
        return s

    # ---- raft_manager.go:142-144
    def StartOnDiskReplica(self, initial_members: dict | None, join: bool, create=None, config: dict | None = None):
        """Register shard config['ShardID'] with its initial members (join = False), or a replica that
        joins an existing shard (join = True, initial_members = None: its ID is mapped when the shard's
        leader recruits it). `create(shardID, replicaID)` is the state machine factory (the engine's
        committed entries reach it through raftd_amd.apply)."""
        self._check_open()
        config = dict(config or {})
        sid = int(config.get("ShardID", 0))
        if join:
            if initial_members:
                raise ErrInvalidOperation("join = true with initial members")
            if sid not in self.shards:
                raise ErrShardNotFound(f"shard {sid}: a joining replica needs the shard started by its members")
            return
        if sid in self.shards:
            raise ErrInvalidOperation(f"shard {sid} already started")
        ids = sorted(int(i) for i in (initial_members or {}))
        want = self.engine_slots(initial_members, self.R)
        have = getattr(self.e, "cfg", {})
        if have and (have.get("initial_members", 0) or (1 << self.R) - 1) != want["initial_members"]:
            raise ErrInvalidOperation("the engine was created for another initial membership "
                                      f"(rg_config.initial_members must be {want['initial_members']:#x})")
        sh = _Shard(ids=[0] * self.R, addrs=[""] * self.R)
        for slot, rid in enumerate(ids):
            sh.ids[slot] = rid
            sh.addrs[slot] = initial_members[rid]
        self.shards[sid] = sh
        if create is not None:
            for rid in ids:
                create(sid, rid)

    # ---- ticking (dragonboat's tick goroutine)
    def tick(self, **inputs):
        self._check_open()
        self.e.tick(**inputs)

    def _members(self, shard_id: int) -> tuple[int, int, int]:
        """(members bits, leader slot or -1, term) as the shard's leader — else its highest-term
        member — knows them."""
        views = [self.e.replica(shard_id * self.R + s) for s in range(self.R)]
        lead = [s for s, v in enumerate(views) if v["role"] == LEADER]
        if lead:
            s = max(lead, key=lambda x: views[x]["term"])
            return views[s]["members"], s, views[s]["term"]
        s = max(range(self.R), key=lambda x: (views[x]["term"], views[x]["members"] != 0))
        return views[s]["members"], -1, views[s]["term"]

    def _sync_change(self, shard_id: int, op: int, slot: int, deadline_ticks: int):
        """Propose a ConfigChange at the leader and tick until the leader applied it."""
        for _ in range(deadline_ticks):
            members, lslot, _ = self._members(shard_id)
            done = bool((members >> slot) & 1) if op == CC_ADD else not (members >> slot) & 1
            if done and lslot >= 0:
                return
            if lslot >= 0 and not self.e.replica(shard_id * self.R + lslot)["cc_pending"]:
                self.e.config_change(shard_id, lslot, op, slot)  # staged for the next tick (once per tick)
            self.tick()
        raise ErrTimeout(f"shard {shard_id}: config change op {op} slot {slot} not applied in {deadline_ticks} ticks")

    # ---- raft_manager.go:165-174 (RecruitReplica)
    def SyncRequestAddReplica(self, shard_id: int, replica_id: int, target: str, config_change_index: int = 0,
                              deadline_ticks: int = 3333):
        sh = self._shard(shard_id)
        if replica_id == 0:
            raise ErrInvalidOperation("replica ID 0")
        if replica_id in sh.removed:
            raise ErrReplicaRemoved(f"replica {replica_id} was removed from shard {shard_id}")
        if replica_id in sh.ids:
            slot = sh.ids.index(replica_id)
            members, _, _ = self._members(shard_id)
            if (members >> slot) & 1:
                return  # already a member
        else:
            members, _, _ = self._members(shard_id)
            free = [s for s in range(self.R) if sh.ids[s] == 0 and not (members >> s) & 1]
            if not free:
                raise ErrRejected(f"shard {shard_id}: every one of the {self.R} replica slots is taken")
            slot = free[0]
            if slot in sh.stale:  # a removed replica lived here: the new one starts as a fresh joiner
                self.e.import_replica(shard_id * self.R + slot, join_view(self.R), [], [], b"")
                sh.stale.discard(slot)
            sh.ids[slot] = replica_id
            sh.addrs[slot] = target
        self._sync_change(shard_id, CC_ADD, slot, deadline_ticks)

    # ---- raft_manager.go:176-185 (RemoveReplica)
    def SyncRequestDeleteReplica(self, shard_id: int, replica_id: int, config_change_index: int = 0,
                                 deadline_ticks: int = 3333):
        sh = self._shard(shard_id)
        if replica_id == 0:  # slot map entries of free slots are 0: never a replica
            raise ErrInvalidOperation("replica ID 0")
        if replica_id not in sh.ids:
            raise ErrRejected(f"replica {replica_id} is not a member of shard {shard_id}")
        slot = sh.ids.index(replica_id)
        self._sync_change(shard_id, CC_REMOVE, slot, deadline_ticks)
        sh.ids[slot] = 0
        sh.addrs[slot] = ""
        sh.removed.add(replica_id)
        sh.stale.add(slot)

    # ---- members.go:21
    def GetLeaderID(self, shard_id: int):
        """(leader replica ID, term, valid): the leader this engine's replicas know (rg_leader)."""
        sh = self._shard(shard_id)
        lid, term, valid = self.e.leader(shard_id)
        if not valid or lid == 0:
            return 0, term, False
        return sh.ids[lid - 1], term, sh.ids[lid - 1] != 0

    # ---- members.go:30
    def SyncGetShardMembership(self, shard_id: int) -> Membership:
        sh = self._shard(shard_id)
        members, _, _ = self._members(shard_id)
        return Membership(nodes={sh.ids[s]: sh.addrs[s] for s in range(self.R) if (members >> s) & 1 and sh.ids[s]},
                          removed=set(sh.removed))

    # ---- raft_manager.go:159
    def Close(self):
        if not self.closed:
            self.closed = True
            close = getattr(self.e, "close", None)
            if close:
                close()
