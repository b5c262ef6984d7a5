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
from raftd_amd.nodehost import (ErrRejected, ErrReplicaRemoved, ErrShardNotFound, NodeHost)

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

    def import_replica(self, rid, view, terms, types=None, payloads=None):
        self.o.import_replica(rid, view, terms, types, payloads)


def scenario(backend):
    nh = NodeHost(backend, R, nhc={"RTTMillisecond": 3, "RaftAddress": "a:63001"})
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
                **NodeHost.engine_slots(MEMBERS, R))


def test_nodehost_over_the_oracle():
    scenario(OracleBackend(**cfg())).Close()


def test_engine_slots():
    assert NodeHost.engine_slots(MEMBERS, 5) == {"initial_members": 0b00111, "join_slots": 0b11000}
    with pytest.raises(Exception):
        NodeHost.engine_slots({}, 5)


@pytest.mark.gpu
def test_nodehost_over_the_engine_matches_the_oracle():
    gpu = make("gpu", **cfg())
    ora = OracleBackend(**cfg())
    gpu.bootstrap()
    scenario(gpu)
    scenario(ora)
    assert gpu.replica_array().tobytes() == ora.replica_array().tobytes()
