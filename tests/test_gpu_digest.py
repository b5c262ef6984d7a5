"""rg_digest against the oracle's or_digest: every replica view and every log entry
(term, type, length, Cmd CRC) of the whole table in one comparison.

- At the bench's own workload (BASELINE metric config, 65,536 groups x 3, 64 x 256-B entries per
  leader per tick, SnapshotEntries 1000): the GPU engine against the oracle of all 65,536 groups,
  through the election, steady state and past the first snapshots / compaction.
- A chaos run (message loss, isolation, caller Cmds of 0..600 bytes through rg_propose with
  max_cmd_bytes 600 > P) where the digest must agree every tick."""
import numpy as np
import pytest

from engines import make

pytestmark = pytest.mark.gpu


def test_digest_full_size_bench_workload():
    G, R, E = 65536, 3, 64
    cfg = dict(groups=G, replicas=R, log_capacity=2048, payload_bytes=256, max_entries_per_msg=E, seed=0x5EED)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
    for e in (gpu, ora):
        e.bootstrap()
    assert gpu.digest() == ora.digest()
    for t in range(26):
        ins = dict(campaign=camp) if t == 1 else dict(prop_target=pt, prop_count=pc) if t >= 6 else {}
        gpu.tick(**ins)
        ora.tick(threads=16, **ins)
        if t in (1, 5, 12, 25):
            assert gpu.digest() == ora.digest(), t
    v = ora.replica(0)
    assert v["snap_index"] >= 1000 and v["marker"] > 0  # the run went past a snapshot and compaction


def test_digest_chaos_every_tick():
    G, R = 48, 3
    cfg = dict(groups=G, replicas=R, log_capacity=256, payload_bytes=64, max_cmd_bytes=600, max_entries_per_msg=8,
               snapshot_entries=30, compaction_overhead=4, drop_ppm=40000, seed=0xD1)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    for e in (gpu, ora):
        e.bootstrap()
    rng = np.random.default_rng(9)
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    for t in range(60):
        batches = []
        if t >= 4:
            for g in range(G):
                if rng.random() < 0.6:
                    n = int(rng.integers(1, 5))
                    batches.append((g, int(rng.integers(0, R)),
                                    [bytes(rng.integers(0, 256, int(rng.integers(0, 601)), dtype=np.uint8))
                                     for _ in range(n)]))
        iso = (rng.random(G * R) < 0.03).astype(np.uint8)
        for e in (gpu, ora):
            if batches:
                e.propose(batches)
            e.tick(campaign=camp if t == 1 else None, isolate=iso)
        assert gpu.digest() == ora.digest(), t
