"""Snapshot events (rg_snapshot_events) against the oracle, tick by tick, and the snapshot host
path (raftd_amd/snapshot.py) driven by the GPU engine end to end: restores and snapshots are
reported at exactly the oracle's indices and terms (single engine, slot filter, four ranks),
and replicas restored from snapshots end with the same application state as their peers."""
import numpy as np
import pytest

from engines import make
from snapshot_helpers import OracleFeeds
from test_snapshot import CFG, run_cluster
from raftd_amd.engine import SNAP_RESTORED, SNAP_TAKEN

pytestmark = pytest.mark.gpu

FIELDS = ("group", "replica_id", "rid", "kind", "restored", "index", "term")


def rows(ev):
    """Event rows by replica id (the device reports them slot by slot)."""
    return sorted(tuple(int(r[f]) for f in FIELDS) for r in ev)


def spells(rng, iso):
    r = rng.random(iso.shape[0])
    return np.where(iso == 1, r >= 0.08, r < 0.015).astype(np.uint8)


def drive(eng, ora, G, R, ticks, seed, check):
    rng = np.random.default_rng(seed)
    iso = np.zeros(G * R, np.uint8)
    seen = {SNAP_RESTORED: 0, SNAP_TAKEN: 0}
    for t in range(ticks):
        pt = rng.integers(0, R, G).astype(np.uint8)
        pt[rng.random(G) < 0.2] = 0xFF
        pc = rng.integers(1, CFG["max_entries_per_msg"] + 1, G).astype(np.uint32)
        camp = (rng.random(G * R) < 0.01).astype(np.uint8)
        iso = spells(rng, iso)
        eng.tick(pt, pc, camp, iso)
        ora.tick(pt, pc, camp, iso)
        want = OracleFeeds(ora, R, CFG["payload_bytes"]).snapshot_events()
        check(t, want)
        for k in seen:
            seen[k] += int(((want["kind"] & k) != 0).sum())
    return seen


@pytest.mark.parametrize("R", [3, 5])
def test_snapshot_events_match_oracle(R):
    G = 8
    cfg = dict(groups=G, replicas=R, seed=61 + R, **CFG)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    gpu.bootstrap()
    ora.bootstrap()

    def check(t, want):
        assert rows(gpu.snapshot_events()) == rows(want), t
        if t % 9 == 0:  # slot filter
            sub = want[(want["replica_id"] == 2)]
            assert rows(gpu.snapshot_events(slot_mask=0b10)) == rows(sub), t
    seen = drive(gpu, ora, G, R, 300, R, check)
    assert seen[SNAP_RESTORED] >= 10 and seen[SNAP_TAKEN] >= 100, seen


def test_snapshot_events_cluster():
    from raftd_amd.cluster import LoopbackCluster
    G, R = 8, 3
    cfg = dict(groups=G, replicas=R, seed=67, **CFG)
    cl, ora = LoopbackCluster(ranks=4, **cfg), make("c", **cfg)
    cl.bootstrap()
    ora.bootstrap()

    def check(t, want):
        assert rows(cl.snapshot_events()) == rows(want), t
    seen = drive(cl, ora, G, R, 200, 5, check)
    assert seen[SNAP_RESTORED] >= 5, seen


def test_snapshot_driver_gpu_end_to_end(tmp_path):
    """One fake application per node behind the GPU engine: restored replicas converge."""
    G, R = 8, 3
    gpu = make("gpu", groups=G, replicas=R, seed=91, **CFG)
    gpu.bootstrap()
    counts, shared = run_cluster(gpu, gpu, lambda rid: gpu.replica(rid)["applied"], G, R, 300, 91, tmp_path)
    assert counts["restored"] >= 10 and counts["taken"] > 100 and shared > 0, counts


def test_snapshot_driver_cluster_end_to_end(tmp_path):
    from raftd_amd.cluster import LoopbackCluster
    G, R = 8, 3
    cl = LoopbackCluster(ranks=4, groups=G, replicas=R, seed=93, **CFG)
    cl.bootstrap()
    counts, shared = run_cluster(cl, cl, lambda rid: cl.replica(rid)["applied"], G, R, 200, 93, tmp_path)
    assert counts["restored"] >= 5 and shared > 0, counts


def test_snapshot_events_full_size():
    """64K groups x 3, SnapshotEntries 1000: every replica snapshots once per ~16 ticks of 64
    entries; each reported snapshot is the replica's snap_index/snap_term after the tick."""
    G, R, E = 65536, 3, 64
    eng = make("gpu", groups=G, replicas=R, log_capacity=2048, payload_bytes=256, max_entries_per_msg=E)
    eng.bootstrap()
    eng.tick()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    eng.tick(campaign=camp)
    pt = np.zeros(G, np.uint8)
    pc = np.full(G, E, np.uint32)
    total = 0
    prev = eng.replica_array()
    for t in range(40):
        eng.tick(pt, pc)
        ev = eng.snapshot_events()
        cur = eng.replica_array()
        want = np.nonzero(cur["snap_index"] != prev["snap_index"])[0]
        assert np.array_equal(np.sort(ev["rid"].astype(np.int64)), want), t
        assert (ev["kind"] == SNAP_TAKEN).all() and (ev["restored"] == 0).all()
        v = cur[ev["rid"].astype(np.int64)]
        assert np.array_equal(ev["index"], v["snap_index"]) and np.array_equal(ev["term"], v["snap_term"])
        assert np.array_equal(v["snap_index"], v["applied"])
        total += len(ev)
        prev = cur
    assert total >= G * R  # each replica snapshotted at least once in 40 ticks
