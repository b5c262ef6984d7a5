"""BASELINE.json configs at full size on the GPU, checked bit-exactly on windows of groups.

Raft groups are independent: an oracle of the groups [base, base + n) (oracle `group_base`) must
reproduce that window of a full-size run — every replica view, outbound message and log entry
with payload. Each test also checks size-independent properties over ALL groups.

- C3: 65,536 groups x 5 replicas spread over 8 ranks (N ranks as N engines on this one GPU, every
  cross-rank message through the wire), 64-entry batches of 256-B entries with CRC32, a 2,048-entry
  log ring and raftd's SnapshotEntries 1000 / CompactionOverhead 5: every replica snapshots and
  compacts twice within the run. The paged payload store holds only live Cmds, so the eight ranks'
  engines fit this one GPU.
- C4: election storm, 65,536 groups x 3, no leader: randomized timeouts, split votes, term bumps;
  10% of the groups start with a follower holding a divergent uncommitted suffix (1-16 entries of
  term 2) and 5% with a second one (term 3), forcing truncation once a leader emerges.
- C5: 1,048,576 groups x 3, Zipf(1.1)-skewed proposals (mean 1 entry per group per tick) with
  snapshot/compaction index advance on the hot groups, 256-B Cmds, L = 2,048, E = 16,
  K = 4. 3.1 M replicas fit one GPU's HBM because payload pages hold only live Cmds.
"""
import zlib

import numpy as np
import pytest

from engines import make

pytestmark = pytest.mark.gpu


NEWEST = 64  # entries compared per replica (the newest; one bulk read each)


def compare_window(view, msgs, entries, ora, base, n, R, t, check_entries=True):
    """view(grid) / msgs(grid, d) / entries(grid, first, count) of the full-size run vs the oracle
    of the window [base, base + n)."""
    for lr in range(n * R):
        gr = base * R + lr
        ov = ora.replica(lr)
        gv = view(gr)
        assert gv == ov, f"tick {t} replica {gr}: " + str({k: (gv[k], ov[k]) for k in ov if gv[k] != ov[k]})
        for d in range(R):
            assert msgs(gr, d) == ora.msgs(lr, d), f"tick {t} msgs {gr}->{d}"
        if check_entries and ov["last"] > ov["marker"]:
            lo = max(ov["marker"] + 1, ov["last"] - NEWEST + 1)
            got = entries(gr, lo, ov["last"] - lo + 1)
            want = [ora.entry(lr, i, with_payload=True) for i in range(lo, ov["last"] + 1)]
            assert got == want, f"tick {t} entries of {gr} from {lo}"


def engine_window_check(eng, ora, base, n, R, t, entries=True):
    views = eng.replicas(base * R, n * R)
    compare_window(lambda gr: views[gr - base * R], eng.msgs,
                   lambda gr, lo, k: eng.entries(gr, lo, k, with_payload=True), ora, base, n, R, t, entries)


def test_c4_election_storm_full_size():
    G, R, W = 65536, 3, 1024
    cfg = dict(replicas=R, log_capacity=256, payload_bytes=16, max_entries_per_msg=16, seed=0xC4)
    eng = make("gpu", groups=G, **cfg)
    wins = [(0, W), (G - W, W)]
    oras = [make("c", groups=n, group_base=b, **cfg) for b, n in wins]
    eng.bootstrap()
    for o in oras:
        o.bootstrap()
    rng = np.random.default_rng(4)
    div1 = np.flatnonzero(rng.random(G) < 0.10)
    div2 = div1[rng.random(len(div1)) < 0.5]
    P = cfg["payload_bytes"]

    def diverge(g, s, term, k):
        v = eng.replica(g * R + s)
        v.update(term=term, vote=0, leader=0, last=R + k)
        terms = [1] * R + [term] * k
        types = [1] * R + [0] * k
        pay = bytes((g * 7 + s * 131 + i) & 0xFF for i in range((R + k) * P))
        eng.import_replica(g * R + s, v, terms, types, pay)
        for (b, n), o in zip(wins, oras):
            if b <= g < b + n:
                o.import_replica((g - b) * R + s, v, terms, types, pay)

    for g in div1:
        diverge(int(g), 1, 2, 1 + int(g) % 16)
    for g in div2:
        diverge(int(g), 2, 3, 1 + (int(g) // 16) % 16)
    pt = np.zeros(G, np.uint8)
    pc = np.full(G, 4, np.uint32)
    for t in range(70):
        ins = dict(prop_target=pt, prop_count=pc) if t >= 45 else {}  # a leader's first entries
        eng.tick(**ins)
        for (b, n), o in zip(wins, oras):
            o.tick(**{k: v[b:b + n] for k, v in ins.items()})
        if t in (12, 25, 44, 69):
            for (b, n), o in zip(wins, oras):
                engine_window_check(eng, o, b, n, R, t, entries=t in (44, 69))
    views = eng.replicas()
    terms = np.array([v["term"] for v in views]).reshape(G, R)
    roles = np.array([v["role"] for v in views]).reshape(G, R)
    assert all(v["err"] == 0 for v in views)
    assert terms.max() >= 4 and np.mean((roles == 2).any(axis=1)) > 0.9  # elections converged
    # truncation happened: many divergent followers' entry 4 no longer carries their term-2 suffix
    e4 = [eng.entry(int(g) * R + 1, R + 1) for g in div1[:400]]
    assert sum(1 for e in e4 if e is not None and e["term"] != 2) > 40


def zipf_rates(G, rng, s=1.1):
    w = 1.0 / np.arange(1, G + 1, dtype=np.float64) ** s
    lam = np.empty(G)
    lam[rng.permutation(G)] = w * (G / w.sum())  # mean 1 entry per group per tick
    return lam


def test_c5_one_million_groups_zipf_compaction():
    G, R, E = 1 << 20, 3, 16
    cfg = dict(replicas=R, log_capacity=2048, payload_bytes=256, max_entries_per_msg=E, max_msgs_per_pair=4,
               snapshot_entries=1000, compaction_overhead=5, seed=0xC5)
    eng = make("gpu", groups=G, **cfg)
    assert eng.device_bytes < 288e9, eng.device_bytes  # the "288 GB HBM sizing" of BASELINE config 5
    rng = np.random.default_rng(5)
    lam = zipf_rates(G, rng)
    hot = int(np.argmax(lam))
    W = 2048
    wins = [(0, W), (min(max(hot - W // 2, 0), G - W), W)]
    oras = [make("c", groups=n, group_base=b, **cfg) for b, n in wins]
    eng.bootstrap()
    for o in oras:
        o.bootstrap()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    props = 0
    for t in range(90):
        ins = {}
        if t == 1:
            ins = dict(campaign=camp)
        elif t >= 6:
            cnt = np.minimum(rng.poisson(lam), E).astype(np.uint32)
            ins = dict(prop_target=np.where(cnt > 0, 0, 0xFF).astype(np.uint8), prop_count=cnt)
            props += int(cnt.sum())
        eng.tick(**ins)
        for (b, n), o in zip(wins, oras):
            o.tick(**{k: v[b * (R if k == "campaign" else 1):(b + n) * (R if k == "campaign" else 1)]
                      for k, v in ins.items()})
        if t in (40, 89):
            for (b, n), o in zip(wins, oras):
                engine_window_check(eng, o, b, n, R, t, entries=(t == 89))
    lead = eng.replicas(hot * R, R)[0]
    assert lead["role"] == 2 and lead["snap_index"] >= 1000 and lead["marker"] > 0  # compaction advanced
    views = eng.replicas(0, 3 * 65536)
    assert all(v["err"] == 0 for v in views)
    for _ in range(3):  # let the last batches commit
        eng.tick()
    committed = eng.sum_committed() - G * (R + 1)  # minus the bootstrap entries and each leader's no-op
    assert 0.98 * props <= committed <= props
    lead = eng.replica(hot * R)
    for s in range(R):
        e = eng.entry(hot * R + s, lead["last"], with_payload=True)
        assert e["crc"] == zlib.crc32(e["payload"]) and e["len"] == 256
    ps = eng.pool_stats()
    assert not ps["failed"] and ps["free"] < ps["total"], ps


def test_c3_five_replicas_eight_ranks_full_size():
    """C3 at its stated size with raftd's snapshot settings: 65,536 groups x 5 spread over 8 ranks,
    64 x 256-B entries per leader per tick, L 2,048, SnapshotEntries 1000, CompactionOverhead 5 —
    every replica snapshots and compacts twice, and every follower entry crosses ranks."""
    from raftd_amd.cluster import LoopbackCluster
    G, R, N, W = 65536, 5, 8, 256
    cfg = dict(replicas=R, log_capacity=2048, payload_bytes=256, max_entries_per_msg=64, snapshot_entries=1000,
               compaction_overhead=5, seed=0xC3)
    # 40,960 replicas per rank, each holding ~1,100 live 256-B Cmds (70 pages) at most
    cl = LoopbackCluster(ranks=N, groups=G, pool_pages=1 << 22, **cfg)
    assert cl.device_bytes < 288e9, cl.device_bytes
    wins = [(0, W), (G - W, W)]
    oras = [make("c", groups=n, group_base=b, **cfg) for b, n in wins]
    cl.bootstrap()
    for o in oras:
        o.bootstrap()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    pt, pc = np.zeros(G, np.uint8), np.full(G, 64, np.uint32)
    for t in range(44):
        ins = dict(campaign=camp) if t == 1 else (dict(prop_target=pt, prop_count=pc) if t >= 6 else {})
        cl.tick(**ins)
        for (b, n), o in zip(wins, oras):
            o.tick(**{k: v[b * (R if k == "campaign" else 1):(b + n) * (R if k == "campaign" else 1)]
                      for k, v in ins.items()}, threads=8)
        if t in (7, 24, 43):
            for (b, n), o in zip(wins, oras):
                compare_window(cl.replica, cl.msgs, lambda gr, lo, k: cl.entries(gr, lo, k, with_payload=True), o,
                               b, n, R, t, check_entries=(t != 7))
    assert cl.wire_bytes > 4 * G * 64 * 256  # every follower entry crossed ranks
    assert cl.sum_committed() >= G * (R + 1 + 36 * 64)  # slot-0 replicas committed the batches
    for g in (0, G // 2 + 3, G - 1):
        for s in range(R):
            v = cl.replica(g * R + s)
            assert v["snap_index"] >= 2000 and v["marker"] == v["snap_index"] - 5 and v["last"] > 2048, v
            assert v["err"] == 0


def test_c2_steady_state_full_shard_set():
    """C2 at its stated size: 4,096 groups x 3, steady-state leaders, 64-entry batches of 256-B
    entries every tick, against the oracle of ALL 4,096 groups — every replica view every tick,
    messages and the newest entries (with payload) on sampled groups — for 48 ticks, past one wrap
    of the 2,048-entry log ring."""
    G, R, E, L = 4096, 3, 64, 2048
    cfg = dict(groups=G, replicas=R, log_capacity=L, payload_bytes=256, max_entries_per_msg=E, seed=0xC2)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    for e in (gpu, ora):
        e.bootstrap()
    for t, ins in enumerate([{}, dict(campaign=camp), {}, {}, {}, {}]):
        gpu.tick(**ins)
        ora.tick(threads=16, **ins)
    pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
    sample = list(range(0, G, 97))
    for t in range(48):
        gpu.tick(pt, pc)
        ora.tick(pt, pc, threads=16)
        ga, oa = gpu.replica_array(), ora.replica_array()
        if ga.tobytes() != oa.tobytes():
            bad = [r for r in range(G * R) if ga[r].tobytes() != oa[r].tobytes()][:3]
            raise AssertionError(f"tick {t}: replicas {bad} differ: {[(gpu.replica(r), ora.replica(r)) for r in bad]}")
        if t % 8 == 7:
            for g in sample:
                for s in range(R):
                    for d in range(R):
                        assert gpu.msgs(g * R + s, d) == ora.msgs(g * R + s, d), (t, g, s, d)
            for g in sample[::4]:
                for s in range(R):
                    v = ora.replica(g * R + s)
                    lo = max(v["marker"] + 1, v["last"] - NEWEST + 1)
                    got = gpu.entries(g * R + s, lo, v["last"] - lo + 1, with_payload=True)
                    assert got == [ora.entry(g * R + s, i, with_payload=True) for i in range(lo, v["last"] + 1)]
    v = gpu.replica_array()
    assert (v["err"] == 0).all() and (v["last"] > L).all()  # every log wrapped the ring
    assert (v["committed"][0::R] >= R + 1 + 46 * E).all()  # slot-0 leaders committed the batches (one in flight)
