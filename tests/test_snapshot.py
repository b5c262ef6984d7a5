"""Snapshot host path (raftd_amd/snapshot.py) against raftd's OnDiskStateMachine snapshot calls
(/root/reference/raft/state_machine.go:186-256) and dragonboat's call order, on the CPU: Go
encoding/json re-marshalling, the three requests byte for byte, the snapshot store, and an
end-to-end run of the oracle with one fake application per node — every replica that restored
from a snapshot ends with the same application state as its peers."""
import os

import numpy as np
import pytest

from engines import make
from snapshot_helpers import NodeApp, OracleFeeds, converged
from raftd_amd.apply import HighStatusCode
from raftd_amd.engine import SNAP_RESTORED, SNAP_TAKEN, SNAPSHOT_EVENT_DTYPE
from raftd_amd.snapshot import (SnapshotDriver, SnapshotStore, go_marshal, go_unmarshal_any, prepare_snapshot,
                                recover_from_snapshot, save_snapshot)


def test_go_marshal_of_decoded_any():
    # json.Unmarshal into any, then json.Marshal: keys sorted, numbers float64, HTML escaping
    v = go_unmarshal_any(b'{"b": 1, "a": [1.50, "<x>&", null, true, false, "\\u00e9\\u2028\\u0001\\t"], "A": {}}')
    assert go_marshal(v) == '{"A":{},"a":[1.5,"\\u003cx\\u003e\\u0026",null,true,false,"é\\u2028\\u0001\\t"],"b":1}'.encode()
    cases = {"0": "0", "-0": "-0", "100": "100", "1e20": "100000000000000000000", "1e21": "1e+21",
             "0.000001": "0.000001", "0.0000001": "1e-7", "1.5e-10": "1.5e-10", "12345678901234567891":
             "12345678901234567000", "0.1": "0.1", "5e-324": "5e-324", "1.7976931348623157e308":
             "1.7976931348623157e+308", "3.0": "3", "-2.5e30": "-2.5e+30"}
    for src, want in cases.items():
        assert go_marshal(go_unmarshal_any(src.encode())) == want.encode(), src
    with pytest.raises(ValueError):
        go_unmarshal_any(b"1e400")  # cannot unmarshal number 1e400 into float64


def test_requests_match_raftd():
    app = NodeApp()
    try:
        prepared = prepare_snapshot(app.url, 7, 2)
        assert prepared == {"Shard": 7.0, "Index": 0.0, "Digest": 0.0}
        data = save_snapshot(app.url, prepared)
        recover_from_snapshot(app.url, data)
        (p1, h1, b1), (p2, h2, b2), (p3, h3, b3) = app.calls
        # PrepareSnapshot: doReqWithContext, raftd headers, no body, no content-type
        assert p1 == "/PrepareSnapshot" and b1 == b"" and h1["content-length"] == "0"
        assert h1["raftd-node-id"] == "7" and h1["raftd-replica-id"] == "2" and "content-type" not in h1
        # SaveSnapshot: json.Marshal(prepared) to /Snapshot, json content-type, no raftd headers
        assert p2 == "/Snapshot" and b2 == b'{"Digest":0,"Index":0,"Shard":7}'
        assert h2["content-type"] == "application/json" and "raftd-node-id" not in h2
        # RecoverFromSnapshot: the raw bytes, octet-stream, no raftd headers
        assert p3 == "/RecoverFromSnapshot" and b3 == data and h3["content-type"] == "application/octet-stream"
        assert "raftd-replica-id" not in h3
        with pytest.raises(HighStatusCode) as ei:
            recover_from_snapshot(app.url + "/nope", b"")
        assert ei.value.status == 404
    finally:
        app.close()


def test_store_keeps_newest_and_detects_damage(tmp_path):
    st = SnapshotStore(str(tmp_path), keep=2)
    for i in (10, 20, 30):
        st.save(5, 1, i, 2, b"data%d" % i)
    assert st.indices(5, 1) == [20, 30]
    assert st.load(5, 1, 30) == (2, b"data30")
    assert st.find(5, 20, 3) == (2, b"data20") and st.find(5, 10, 3) is None and st.find(6, 20, 3) is None
    path = os.path.join(str(tmp_path), "%016x" % 5, "1", "%016x" % 30)
    raw = bytearray(open(path, "rb").read())
    raw[-1] ^= 1
    open(path, "wb").write(bytes(raw))
    with pytest.raises(ValueError):
        st.load(5, 1, 30)


class FakeFeeds:
    def __init__(self, events, recs, pay):
        self.ev, self.recs, self.pay = events, recs, pay

    def snapshot_events(self, slot_mask=0xFF):
        return self.ev

    def apply_committed(self, slot_mask=0xFF):
        return self.recs, self.pay


def test_driver_orders_calls_per_replica(tmp_path):
    from test_apply import fake_batch
    recs, pay = fake_batch()  # rid 4 (shard 3, replica 2): indices 7..9; rid 9 (shard 17, replica 1): 12..13
    ev = np.array([(3, 2, 4, SNAP_RESTORED | SNAP_TAKEN, 0, 6, 9, 4), (17, 1, 9, SNAP_TAKEN, 0, 0, 13, 5)],
                  SNAPSHOT_EVENT_DTYPE)
    apps = {r: NodeApp() for r in (1, 2)}
    st = SnapshotStore(str(tmp_path))
    st.save(3, 1, 6, 4, b"\x03\0\0\0\0\0\0\0\x06\0\0\0\0\0\0\0\x2a\0\0\0")  # leader's snapshot at 6
    drv = SnapshotDriver({r: a.url for r, a in apps.items()}, st, replicas=3)
    try:
        out = drv.after_tick(FakeFeeds(ev, recs, pay))
        assert [rt.calls for rt in out] == [
            [("RecoverFromSnapshot", 6), ("Update", 7, 9), ("SaveSnapshot", 9)],
            [("Update", 12, 13), ("SaveSnapshot", 13)]]
        assert [c[0] for c in apps[2].calls] == ["/RecoverFromSnapshot", "/UpdateEntries", "/PrepareSnapshot", "/Snapshot"]
        assert st.indices(3, 2) == [6, 9] and st.indices(17, 1) == [13]  # the received copy is kept
        assert st.load(3, 2, 9)[0] == 4
        with pytest.raises(LookupError):  # a restore with no snapshot anywhere
            drv.after_tick(FakeFeeds(np.array([(3, 3, 5, SNAP_RESTORED, 0, 99, 0, 0)], SNAPSHOT_EVENT_DTYPE),
                                     recs[:0], pay[:0]))
    finally:
        drv.close()
        for a in apps.values():
            a.close()


CFG = dict(log_capacity=64, payload_bytes=16, max_entries_per_msg=8, snapshot_entries=12, compaction_overhead=3,
           drop_ppm=100000)


def run_cluster(eng, feeds, applied_of, G, R, ticks, seed, tmp_path, on_tick=None):
    """Tick `eng` with random inputs (followers isolated for stretches, so they fall behind the
    leader's compaction marker), driving one fake application per node after every tick."""
    rng = np.random.default_rng(seed)
    apps = {r: NodeApp() for r in range(1, R + 1)}
    drv = SnapshotDriver({r: a.url for r, a in apps.items()}, SnapshotStore(str(tmp_path)), replicas=R)
    counts = {"restored": 0, "taken": 0, "updates": 0}
    iso = np.zeros(G * R, np.uint8)
    try:
        for t in range(ticks):
            pt = rng.integers(0, R, G).astype(np.uint8)
            pt[rng.random(G) < 0.2] = 0xFF
            pc = rng.integers(1, 9, G).astype(np.uint32)
            camp = (rng.random(G * R) < 0.01).astype(np.uint8)
            # isolation spells: a replica is cut off for ~12 ticks at a time (~16% of replicas)
            r = rng.random(G * R)
            iso = np.where(iso == 1, r >= 0.08, r < 0.015).astype(np.uint8)
            eng.tick(pt, pc, camp, iso)
            if on_tick:
                on_tick(t)
            for rt in drv.after_tick(feeds):
                counts["restored"] += bool(rt.restored)
                counts["taken"] += rt.snapshot is not None
                counts["updates"] += rt.update is not None
        shared = converged([apps[r] for r in range(1, R + 1)], applied_of, G, R)
    finally:
        drv.close()
        for a in apps.values():
            a.close()
    return counts, shared


def test_oracle_end_to_end_snapshots_converge(tmp_path):
    G, R = 6, 3
    ora = make("c", groups=G, replicas=R, seed=91, **CFG)
    ora.bootstrap()
    counts, shared = run_cluster(ora, OracleFeeds(ora, R, CFG["payload_bytes"]),
                                 lambda rid: ora.replica(rid)["applied"], G, R, 400, 91, tmp_path)
    assert counts["restored"] >= 20 and counts["taken"] > 200 and counts["updates"] > 600, counts
    assert shared > 0
