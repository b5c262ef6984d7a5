"""Crash and restart through the host WAL: every tick the engine's persistence feed
(rg_persist_collect) is appended to a node-local WAL and fsynced; mid-run the engine is dropped,
the WAL replayed, and (1) the replayed hard state and log equal what the engine held (terms,
types, lengths, CRCs, payloads), (2) an engine restored from it and an oracle restored the same
way then run bit-identically, single engine and two ranks (one WAL per node)."""
import numpy as np
import pytest

from engines import make
from test_gpu_parity import CHAOS, compare, random_inputs

pytestmark = pytest.mark.gpu


def check_replayed(eng, logs, rids):
    for rid, gr in rids:
        v = eng.replica(rid)
        s = logs[gr].state
        assert (s["term"], s["vote"], s["commit"], s["last"], s["marker"]) == \
            (v["term"], v["vote"], v["committed"], v["last"], v["marker"]), gr
        if v["last"] > v["marker"]:
            got = eng.entries(rid, v["marker"] + 1, v["last"] - v["marker"], with_payload=True)
            want = [dict(term=t, type=ty, len=ln, crc=c, payload=p)
                    for t, ty, ln, c, p in (logs[gr].log[i] for i in range(v["marker"] + 1, v["last"] + 1))]
            assert got == want, gr


@pytest.mark.parametrize("ranks", [1, 2])
def test_crash_restart_from_wal(tmp_path, ranks):
    from raftd_amd.wal import WAL, replay, restore
    cfg = dict(groups=6, replicas=3, seed=61, **dict(CHAOS, snapshot_entries=15))
    full = dict(CHAOS, snapshot_entries=15, replicas=3, seed=61, election_rtt=10, heartbeat_rtt=1)
    if ranks == 1:
        engines = [make("gpu", **cfg)]
    else:
        from raftd_amd.cluster import LoopbackCluster
        cl = LoopbackCluster(ranks=ranks, **cfg)
        engines = cl.engines
    for e in engines:
        e.bootstrap()
    wals = [WAL(str(tmp_path / f"node{k}.wal")) for k in range(len(engines))]
    for k, e in enumerate(engines):  # the bootstrap state: a checkpoint record
        wals[k].append(0, *e.persist_collect(full=True), cfg["payload_bytes"])
    rng = np.random.default_rng(62)
    G, R = cfg["groups"], cfg["replicas"]
    for t in range(70):
        ins = random_inputs(rng, G, R, cfg["max_entries_per_msg"])
        (engines[0] if ranks == 1 else cl).tick(*ins)
        for k, e in enumerate(engines):
            wals[k].append(t + 1, *e.persist_collect(), cfg["payload_bytes"])
    rids = [[(lr, e.global_id(lr)[1]) for lr in range(e.nrep)] for e in engines]
    logs = [replay(w.path, R) for w in wals]
    for e, lg, rr in zip(engines, logs, rids):
        check_replayed(e, lg, rr)
    # crash: every node restarts from its own WAL; an oracle restarts from all of them
    gpu = make("gpu", **cfg) if ranks == 1 else LoopbackCluster(ranks=ranks, **cfg)
    ora = make("c", **cfg)
    gpu.bootstrap()
    ora.bootstrap()
    new = [gpu] if ranks == 1 else gpu.engines
    for e, lg, rr in zip(new, logs, rids):
        restore(e, lg, dict(cfg, **full), rr)
        restore(ora, lg, dict(cfg, **full), [(gr, gr) for _, gr in rr])
    compare(gpu, ora, -1)
    for t in range(60):
        ins = random_inputs(rng, G, R, cfg["max_entries_per_msg"])
        gpu.tick(*ins)
        ora.tick(*ins)
        compare(gpu, ora, t)
    assert max(gpu.replica(r)["committed"] for r in range(G * R)) > 60
