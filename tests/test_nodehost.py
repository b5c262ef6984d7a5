"""raftd_amd.nodehost: the NodeHost subset raftd calls (raft/raft_manager.go:142-184, raft/members.go:21-30)
over the engine, with raftd's arbitrary replica IDs mapped onto the engine's slots.

The same scenario runs on the C oracle (CPU; the oracle only stands in for the engine behind the shim
here, as test infrastructure) and on the GPU engine (`-m gpu`), where every replica is then compared
with the oracle run bit for bit: initial members 10/20/30 of five slots, an election, RecruitReplica
of 40 into a join slot, RemoveReplica of 20, the removed ID refused, 50 and 60 recruited (60 into the
slot 20 left, reset to a fresh joiner first), a sixth member refused, and a second shard untouched."""
import numpy as np
import pytest

from engines import make
from raftd_amd.nodehost import (ColocatedNodeHost, ErrRejected, ErrReplicaRemoved, ErrShardNotFound)

R = 5
MEMBERS = {30: "c:63001", 10: "a:63001", 20: "b:63001"}


class OracleBackend:
    """The engine's interface over the C oracle (tests only)."""

    def __init__(self, **cfg):
        self.o = make("c", **cfg)
        self.o.bootstrap()
        self.cfg = self.o.cfg

    def tick(self, **kw):
        self.o.tick(**kw)

    def replica(self, rid):
        return self.o.replica(rid)

    def replica_array(self):
        return self.o.replica_array()

    def config_change(self, group, slot, op, target):
        rc = self.o.config_change(group, slot, op, target)
        if rc:
            raise RuntimeError(f"or_config_change: {rc}")

    def leader(self, group):
        views = [self.o.replica(group * R + s) for s in range(R)]
        lead = [s for s, v in enumerate(views) if v["role"] == 2]
        if not lead:
            return 0, max(v["term"] for v in views), False
        s = max(lead, key=lambda x: views[x]["term"])
        return s + 1, views[s]["term"], True

    def import_replica(self, rid, view, terms, types=None, payloads=None, lens=None):
        self.o.import_replica(rid, view, terms, types, payloads, lens)

    @property
    def t(self):
        return self.o.t


def scenario(backend):
    nh = ColocatedNodeHost(backend, R, nhc={"RTTMillisecond": 3, "RaftAddress": "a:63001"})
    created = []
    for sid in (0, 1):
        nh.StartOnDiskReplica(MEMBERS, False, lambda s, r: created.append((s, r)), {"ShardID": sid, "ReplicaID": 10})
    assert sorted(created) == [(0, 10), (0, 20), (0, 30), (1, 10), (1, 20), (1, 30)]
    camp = np.zeros(2 * R, np.uint8)
    camp[0::R] = 1
    nh.tick()
    nh.tick(campaign=camp)
    for _ in range(4):
        nh.tick()
    lid, term, valid = nh.GetLeaderID(0)
    assert (lid, valid) == (10, True) and term >= 2
    assert nh.SyncGetShardMembership(0).nodes == MEMBERS
    nh.SyncRequestAddReplica(0, 40, "d:63001")
    assert nh.SyncGetShardMembership(0).nodes == {**MEMBERS, 40: "d:63001"}
    nh.SyncRequestDeleteReplica(0, 20)
    m = nh.SyncGetShardMembership(0)
    assert m.nodes == {10: "a:63001", 30: "c:63001", 40: "d:63001"} and m.removed == {20}
    with pytest.raises(ErrReplicaRemoved):
        nh.SyncRequestAddReplica(0, 20, "b:63001")
    nh.SyncRequestAddReplica(0, 50, "e:63001")  # the last join slot
    nh.SyncRequestAddReplica(0, 60, "f:63001")  # slot 1, where 20 lived: reset to a fresh joiner first
    assert set(nh.SyncGetShardMembership(0).nodes) == {10, 30, 40, 50, 60}
    with pytest.raises(ErrRejected):
        nh.SyncRequestAddReplica(0, 70, "g:63001")
    for _ in range(12):  # the recruits catch up
        nh.tick()
    lead = backend.replica(0 * R + 0)
    for slot in (1, 3, 4):
        v = backend.replica(0 * R + slot)
        assert v["last"] == lead["last"] and v["committed"] == lead["committed"] and v["term"] == lead["term"], slot
    assert nh.SyncGetShardMembership(1).nodes == MEMBERS  # the other shard never changed
    assert nh.GetLeaderID(1)[:3:2] == (10, True)
    with pytest.raises(ErrShardNotFound):
        nh.GetLeaderID(7)
    return nh


def cfg():
    return dict(groups=2, replicas=R, log_capacity=256, payload_bytes=16, max_entries_per_msg=8, seed=0x7E,
                **ColocatedNodeHost.engine_slots(MEMBERS, R))


def test_nodehost_over_the_oracle():
    scenario(OracleBackend(**cfg())).Close()


def test_engine_slots():
    assert ColocatedNodeHost.engine_slots(MEMBERS, 5) == {"initial_members": 0b00111, "join_slots": 0b11000}
    with pytest.raises(Exception):
        ColocatedNodeHost.engine_slots({}, 5)


@pytest.mark.gpu
def test_nodehost_over_the_engine_matches_the_oracle():
    gpu = make("gpu", **cfg())
    ora = OracleBackend(**cfg())
    gpu.bootstrap()
    scenario(gpu)
    scenario(ora)
    assert gpu.replica_array().tobytes() == ora.replica_array().tobytes()


# ---------------------------------------------------------------- one NodeHost per node
DIRECTORY = [(11, "n0:63001"), (22, "n1:63001"), (33, "n2:63001")]  # rank -> (raftd ReplicaID, address)


def per_node_scenario(backend, G, ticks=160, check=None):
    """One NodeHost per node (rank) over a cluster of every shard (the spread placement, N = R = 3):
    nodes 11 and 22 start their replica of each shard as initial members, node 33 with join = true
    (raft_manager.go:134-144). After the elections node 11 recruits 33 into every shard and node 22
    removes 11 from the even shards, each request proposed at the caller's own replica (a follower
    forwards it) and complete once the caller's replica applied it; GetLeaderID and
    SyncGetShardMembership answer from each node's own replica. check(t) runs after every tick."""
    from raftd_amd.cluster import RankView
    from raftd_amd.nodehost import NodeHost
    N = len(DIRECTORY)
    nhs = [NodeHost(RankView(backend, k, N, N), N, DIRECTORY) for k in range(N)]
    initial = {i: a for i, a in DIRECTORY[:2]}
    for nh in nhs:
        for g in range(G):
            join = nh.replica_id not in initial
            nh.StartOnDiskReplica(None if join else initial, join, None, {"ShardID": g})
    reqs = {}
    for t in range(ticks):
        if t == 40:
            reqs["add"] = [nhs[0].RequestAddReplica(g, 33, "n2:63001", deadline_ticks=80) for g in range(G)]
        if t == 90:
            reqs["del"] = [nhs[1].RequestDeleteReplica(g, 11, deadline_ticks=60) for g in range(0, G, 2)]
        for nh in nhs:
            nh.before_tick()
        backend.tick()
        for nh in nhs:
            nh.after_tick()
        if check:
            check(t, nhs)
    assert all(r.done for r in reqs["add"]), [(r.shard, r.error) for r in reqs["add"] if not r.done]
    assert all(r.done for r in reqs["del"]), [(r.shard, r.error) for r in reqs["del"] if not r.done]
    for g in range(G):
        want = {22: "n1:63001", 33: "n2:63001"} if g % 2 == 0 else dict(DIRECTORY)
        for nh in nhs[1:]:  # node 11 left the even shards: its own replica never learns the removal
            assert nh.SyncGetShardMembership(g).nodes == want, (g, nh.replica_id)
        lid = [nh.GetLeaderID(g) for nh in nhs[1:]]
        assert lid[0][2] and lid[0][0] == lid[1][0] and lid[0][0] in want, (g, lid)
    assert nhs[1].SyncGetShardMembership(0).removed == {11}
    with pytest.raises(ErrReplicaRemoved):
        nhs[1].RequestAddReplica(0, 11, "n0:63001")
    with pytest.raises(ErrRejected):
        nhs[0].RequestAddReplica(1, 44, "n3:63001")  # no such node
    return nhs


def per_node_cfg(G):
    return dict(groups=G, replicas=3, log_capacity=128, payload_bytes=16, max_entries_per_msg=8, snapshot_entries=40,
                compaction_overhead=4, drop_ppm=20000, seed=0x90DE)


def test_nodehost_per_node_over_the_oracle():
    G = 6
    ora = OracleBackend(**per_node_cfg(G))
    per_node_scenario(ora, G)


@pytest.mark.gpu
def test_nodehost_per_node_over_loopback_ranks_matches_the_oracle():
    """The per-node scenario over three ranks (LoopbackCluster: every cross-rank message through the
    wire), every replica bit-exact with the oracle of the whole shard set after every tick."""
    from raftd_amd.cluster import LoopbackCluster
    G = 6
    cl = LoopbackCluster(ranks=3, **per_node_cfg(G))
    cl.bootstrap()
    ora = OracleBackend(**per_node_cfg(G))
    staged, views = [], []

    def check(t, nhs):
        staged.append([x for nh in nhs for x in nh.staged])
        views.append(cl.replicas())

    per_node_scenario(cl, G, check=check)
    # the oracle replays the same starts and the same staged membership inputs, tick by tick
    from raftd_amd.cluster import RankView
    from raftd_amd.nodehost import NodeHost
    nhs = [NodeHost(RankView(ora, k, 3, 3), 3, DIRECTORY) for k in range(3)]
    initial = {i: a for i, a in DIRECTORY[:2]}
    for nh in nhs:
        for g in range(G):
            join = nh.replica_id not in initial
            nh.StartOnDiskReplica(None if join else initial, join, None, {"ShardID": g})
    for t, st in enumerate(staged):
        for g, s, op, target in st:
            ora.config_change(g, s, op, target)
        ora.tick()
        for rid in range(G * 3):
            assert views[t][rid] == ora.replica(rid), (t, rid)
    assert sum(len(s) for s in staged) >= G + G // 2  # every request was proposed


@pytest.mark.gpu
@pytest.mark.parametrize("n,port", [(2, 29541), (3, 29542)])
def test_nodehost_one_per_process_gloo(n, port):
    """One NodeHost per process (rank = node, gloo between them, one GPU): each node starts its own
    replicas (join decided per node), recruit and remove run through the nodes' own replicas, every
    replica bit-exact with the oracle of the whole shard set every tick."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    out = subprocess.run([sys.executable, "-u", os.path.join(here, "nodehost_worker.py"), str(n)], env=env,
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "nodehost parity ok" in out.stdout
