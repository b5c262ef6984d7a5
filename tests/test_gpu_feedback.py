"""Applied-index feedback (rg_notify_applied ≈ dragonboat's Peer.NotifyRaftLastApplied) and the
restart replay it enables, against the oracle.

raftd's on-disk state machine applies asynchronously and, on restart, Open returns the app's
/LastLogIndex (/root/reference/raft/state_machine.go:101-124): entries the WAL holds as committed
but the app never applied are handed to Update again. With rg_config.apply_feedback = 1 the
engine's `applied` moves only when the host reports it; a lagging state machine then delays
campaigns (hasConfigChangeToApply) and snapshots exactly as in the oracle.
"""
import numpy as np
import pytest

from engines import make
from test_gpu_parity import CHAOS, compare, random_inputs
from test_gpu_propose import check_applied
from test_oracle import lagging_apply, random_batches

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("R", [3, 5])
def test_lagging_state_machine(R):
    cfg = dict(CHAOS, groups=4, replicas=R, payload_bytes=64, max_entries_per_msg=8, seed=70 + R, apply_feedback=1)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    gpu.bootstrap()
    ora.bootstrap()
    rng = np.random.default_rng(R)
    G = cfg["groups"]
    lag = 0
    for t in range(120):
        notes = lagging_apply(rng, ora, G * R)
        if notes:
            rids, idx = zip(*notes)
            gpu.notify_applied(list(rids), list(idx))
            for r, i in notes:
                assert ora.notify_applied(r, i) == 0
        b = random_batches(rng, G, R, 8, 64)
        gpu.propose(b)
        ora.propose(b)
        camp = (rng.random(G * R) < 0.03).astype(np.uint8)
        iso = (rng.random(G * R) < 0.05).astype(np.uint8)
        gpu.tick(None, None, camp, iso)
        ora.tick(None, None, camp, iso)
        compare(gpu, ora, t)
        check_applied(gpu, ora)
        lag += sum(1 for r in range(G * R) if ora.replica(r)["applied"] < ora.replica(r)["committed"])
    assert lag > 0


def test_notify_applied_rejects_past_processed():
    from raftd_amd.engine import RgError
    gpu = make("gpu", groups=2, replicas=3, payload_bytes=16, apply_feedback=1)
    gpu.bootstrap()
    gpu.tick()
    v = gpu.replica(1)
    with pytest.raises(RgError):
        gpu.notify_applied([1, 2], [v["processed"], v["processed"] + 1])
    assert gpu.replica(1)["applied"] == v["applied"]  # all or nothing
    gpu.notify_applied([1], [v["processed"]])
    assert gpu.replica(1)["applied"] == v["processed"]


def test_restart_hands_unapplied_entries_to_update(tmp_path):
    """a crash after the WAL fsync but before the tick's /UpdateEntries POSTs.
    The restarted engine starts from the app's applied index and its first tick hands over exactly
    the entries the app missed; an oracle restored the same way agrees tick by tick."""
    from raftd_amd.wal import WAL, replay, restore
    cfg = dict(groups=4, replicas=3, seed=91, **dict(CHAOS, snapshot_entries=30, drop_ppm=0))
    full = dict(cfg, election_rtt=10, heartbeat_rtt=1)
    eng = make("gpu", **cfg)
    eng.bootstrap()
    wal = WAL(str(tmp_path / "node.wal"))
    wal.append(0, *eng.persist_collect(full=True), cfg["payload_bytes"])
    G, R = cfg["groups"], cfg["replicas"]
    app = {}          # global rid -> [(index, Cmd)] the app applied
    rng = np.random.default_rng(5)
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    missed = None
    for t in range(40):
        if t > 1:
            eng.propose(random_batches(rng, G, R, 8, 16, p_none=0.0))
        eng.tick(campaign=camp if t == 1 else None)
        wal.append(t + 1, *eng.persist_collect(), cfg["payload_bytes"])  # fsynced before the POSTs
        recs, pay = eng.apply_committed()
        batch = {}
        for r, p in zip(recs, pay):
            batch.setdefault(int(r["rid"]), []).append((int(r["index"]), bytes(p[:int(r["len"])])))
        if t == 39:  # crash: this tick's POSTs never happen
            missed = batch
            break
        for rid, es in batch.items():
            app.setdefault(rid, []).extend(es)
    assert missed and sum(len(v) for v in missed.values()) > 0
    last_applied = {}
    for rid in range(G * R):
        es = app.get(rid, [])
        last_applied[rid] = es[-1][0] if es else 0
    logs = replay(wal.path, R)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    gpu.bootstrap()
    ora.bootstrap()
    rids = [(r, r) for r in range(G * R)]
    # the app's /LastLogIndex: the last index it applied (application entries only; the restart
    # clamps it to the snapshot index, whose state the app recovers first)
    restore(gpu, logs, full, rids, app_applied=lambda gr: last_applied[gr])
    restore(ora, logs, full, rids, app_applied=lambda gr: last_applied[gr])
    compare(gpu, ora, -1)
    gpu.tick()
    ora.tick()
    compare(gpu, ora, 0)
    check_applied(gpu, ora)
    recs, pay = gpu.apply_committed()
    again = {}
    for r, p in zip(recs, pay):
        again.setdefault(int(r["rid"]), []).append((int(r["index"]), bytes(p[:int(r["len"])])))
    for rid in range(G * R):  # exactly what the app missed (nothing it already had, nothing lost);
        # a snapshot at or past them at the crash covers them instead (RecoverFromSnapshot)
        floor = max(last_applied[rid], logs[rid].state["snap_index"])
        want = [e for e in missed.get(rid, []) if e[0] > floor]
        assert again.get(rid, []) == want, rid
