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


class NodeHost:
    """dragonboat.NodeHost's subset over one engine that hosts every replica of its shards (the
    co-located layout; with ranks, the rank's replicas). `engine` is a raftd_amd.engine.Engine (or
    any object with its tick / config_change / leader / replica / import_replica methods)."""

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
