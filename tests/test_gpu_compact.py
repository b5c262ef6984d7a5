"""rg_compact on the GPU engine against the C oracle's or_compact: between ticks random
shards compact to random indices (capped at each replica's snapshot index), every tick bit-exact —
replicas, messages, entries and payloads — including the InstallSnapshot traffic compaction causes
and the payload pages released below the new marker."""
import numpy as np
import pytest

from engines import make
from test_gpu_parity import CHAOS, check_payloads, compare, random_inputs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("R,seed", [(3, 1), (5, 2)])
def test_compact_matches_oracle(R, seed):
    from raftd_amd import RgError
    G = 24
    cfg = dict(CHAOS, groups=G, replicas=R, snapshot_entries=12, seed=900 + seed)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    gpu.bootstrap()
    ora.bootstrap()
    rng = np.random.default_rng(seed)
    moved = 0
    for t in range(100):
        for g in range(G):
            if rng.random() < 0.25:
                idx = int(rng.integers(0, ora.replica(g * R)["committed"] + 6))
                n = gpu.compact(g, idx)
                assert n == ora.compact(g, idx), (t, g, idx)
                moved += n
        ins = random_inputs(rng, G, R, CHAOS["max_entries_per_msg"])
        gpu.tick(*ins)
        ora.tick(*ins)
        compare(gpu, ora, t)
    check_payloads(gpu, ora)
    assert moved > 50
    with pytest.raises(RgError, match="outside"):
        gpu.compact(G, 1)


def test_compact_releases_pages():
    """With a large CompactionOverhead every replica keeps 60 entries below its snapshot; compacting
    every shard to its snapshot index returns the stream pages below to the pool at the next tick."""
    G, R, E = 8, 3, 16
    cfg = dict(groups=G, replicas=R, log_capacity=256, payload_bytes=256, max_entries_per_msg=E,
               snapshot_entries=64, compaction_overhead=60, seed=5)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    for e in (gpu, ora):
        e.bootstrap()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
    for t in range(30):
        ins = (None, None, camp) if t == 1 else (pt, pc) if t >= 4 else ()
        gpu.tick(*ins)
        ora.tick(*ins)
    before = gpu.pool_stats()["free"]
    for g in range(G):
        snap = ora.replica(g * R)["snap_index"]
        assert snap > ora.replica(g * R)["marker"]
        assert gpu.compact(g, snap) == ora.compact(g, snap) == R
    for _ in range(2):
        gpu.tick()
        ora.tick()
    compare(gpu, ora, "after")
    assert gpu.pool_stats()["free"] > before
