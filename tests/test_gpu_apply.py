"""Committed-entry copy-back (rg_apply_committed) against the oracle's applied entries: after
every tick, each replica's non-empty application entries of (applied before, applied after],
snapshot-restored ranges excluded — index, length, CRC and payload bytes — single engine and
across ranks."""
import zlib

import numpy as np
import pytest

from engines import make
from test_gpu_parity import CHAOS, random_inputs

pytestmark = pytest.mark.gpu


def expected(ora, rids):
    out = []
    for rid in rids:
        out += [(rid, i, ln, crc, p) for i, ln, crc, p in ora.applied_entries(rid)]
    return out


def got(recs, pay, to_global):
    return [(to_global(int(r["rid"])), int(r["index"]), int(r["len"]), int(r["crc"]), bytes(pay[k, :int(r["len"])]))
            for k, r in enumerate(recs)]


def test_apply_copyback_chaos():
    cfg = dict(groups=6, replicas=3, seed=41, **dict(CHAOS, snapshot_entries=15))
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    gpu.bootstrap()
    ora.bootstrap()
    rng = np.random.default_rng(41)
    total = 0
    for t in range(120):
        ins = random_inputs(rng, 6, 3, cfg["max_entries_per_msg"])
        gpu.tick(*ins)
        ora.tick(*ins)
        recs, pay = gpu.apply_committed()
        g = got(recs, pay, lambda rid: rid)
        assert sorted(g) == sorted(expected(ora, range(18))), t
        for (_, _, ln, crc, p) in g:
            assert crc == zlib.crc32(p) and ln == len(p)
        total += len(g)
        if t % 7 == 0:  # a slot filter: only slot-1 replicas
            r1, p1 = gpu.apply_committed(slot_mask=0b010)
            assert sorted(got(r1, p1, lambda rid: rid)) == sorted(expected(ora, range(1, 18, 3)))
    assert total > 500


def test_apply_copyback_cluster():
    from raftd_amd.cluster import LoopbackCluster
    cfg = dict(groups=8, replicas=3, seed=43, **dict(CHAOS, snapshot_entries=15))
    cl, ora = LoopbackCluster(ranks=4, **cfg), make("c", **cfg)
    cl.bootstrap()
    ora.bootstrap()
    rng = np.random.default_rng(43)
    for t in range(80):
        ins = random_inputs(rng, 8, 3, cfg["max_entries_per_msg"])
        cl.tick(*ins)
        ora.tick(*ins)
        allg = []
        for e in cl.engines:
            recs, pay = e.apply_committed()
            allg += got(recs, pay, lambda rid, e=e: e.global_id(rid)[1])
            assert all(int(r["group"]) * 3 + int(r["replica_id"]) - 1 == e.global_id(int(r["rid"]))[1] for r in recs)
        assert sorted(allg) == sorted(expected(ora, range(24))), t


def test_apply_copyback_full_size():
    """64K groups x 3 steady state: every replica applies its 64 entries each tick; spot-check the
    copied payload CRCs against zlib."""
    G, R, E = 65536, 3, 64
    eng = make("gpu", groups=G, replicas=R, log_capacity=2048, payload_bytes=256, max_entries_per_msg=E)
    eng.bootstrap()
    eng.tick()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    eng.tick(campaign=camp)
    for _ in range(4):
        eng.tick()
    pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
    for _ in range(4):
        eng.tick(pt, pc)
    recs, pay = eng.apply_committed(slot_mask=0b001)  # the node hosting every slot-0 replica
    assert len(recs) == G * E
    assert np.all(np.diff(recs["index"].reshape(G, E), axis=1) == 1)
    for k in range(0, len(recs), 9973):
        assert int(recs[k]["crc"]) == zlib.crc32(bytes(pay[k]))


@pytest.mark.parametrize("d2h", ["kernel", "sdma"])
def test_async_copyback_matches_sync(d2h, monkeypatch):
    """rg_apply_async / rg_apply_wait (double-buffered, copy stream) return exactly what
    rg_apply_committed returns for the same tick, also when a buffer is re-used two ticks later —
    with the copy kernel (default) and with the D2H leg on an SDMA engine (RAFTGPU_APPLY_SDMA=1)."""
    from test_gpu_parity import CHAOS, random_inputs
    if d2h == "sdma":
        monkeypatch.setenv("RAFTGPU_APPLY_SDMA", "1")  # read by rg_create
    cfg = dict(CHAOS, groups=8, replicas=3, payload_bytes=64, max_entries_per_msg=16, seed=4)
    eng = make("gpu", **cfg)
    eng.bootstrap()
    rng = np.random.default_rng(4)
    total = 0
    for t in range(60):
        eng.tick(*random_inputs(rng, 8, 3, 16))
        want_r, want_p = eng.apply_committed()
        eng.apply_async(0xFF, t & 1)
        if t % 5 == 4:  # sometimes read the other buffer first: it must still hold the previous tick
            eng.apply_wait((t - 1) & 1)
        got_r, got_p = eng.apply_wait(t & 1)
        assert np.array_equal(got_r, want_r), t
        for k in range(len(want_r)):
            n = int(want_r[k]["len"])
            assert bytes(got_p[k, :n]) == bytes(want_p[k, :n]), (t, k)
        total += len(want_r)
    assert total > 0


def test_apply_batch_ships_runs():
    """The copy-back is ranges (r05): one rg_apply_run per run of consecutive applied indices, 8 B of
    {len, crc} per entry. In steady state every replica's window is one run; the runs are maximal (no
    two runs of a replica touch), their counts tile the per-entry array, and expanding them gives the
    oracle's applied entries exactly."""
    G, R, E = 32, 3, 16
    cfg = dict(groups=G, replicas=R, log_capacity=256, payload_bytes=64, max_entries_per_msg=E, snapshot_entries=0,
               seed=47)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    gpu.bootstrap()
    ora.bootstrap()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
    for t in range(12):
        ins = (None, None, camp) if t == 1 else (pt, pc) if t >= 4 else ()
        gpu.tick(*ins)
        ora.tick(*ins)
        runs, cmds, pay = gpu.apply_batch()
        assert int(runs["count"].sum()) == len(cmds)
        assert np.array_equal(np.cumsum(runs["count"])[:-1] if len(runs) else [], runs["entry"][1:])
        for a, b in zip(runs[:-1], runs[1:]):  # maximal: a replica's next run starts past a gap
            assert a["rid"] != b["rid"] or b["first"] > a["first"] + a["count"]
        if t >= 9:  # steady: every replica's window is one run (followers' windows lag their leader's)
            assert len(runs) == G * R and np.all(runs["count"] >= E), (t, len(runs), runs["count"])
        recs, rows = gpu.apply_committed()
        assert sorted(got(recs, rows, lambda rid: rid)) == sorted(expected(ora, range(G * R))), t
