"""ReadIndex (rg_read_index / rg_read_index_results) against the oracle, tick by tick.

raftd's /raft/get and /raft/GetValue handlers read through the shard with SyncRead
(/root/reference/raft/api.go; dragonboat NodeHost.SyncRead → ReadIndex, Raft thesis §6.4): the
leader records its commit index under the request's context, confirms leadership with a heartbeat
round carrying the context, and the read is ready once a quorum acknowledged it; followers forward
the request and receive a ReadIndexResp. Every replica view, message and ready read (ctx, index)
must equal the oracle's. Parity with dragonboat itself is unpinned.
"""
import numpy as np
import pytest

from engines import make
from test_gpu_parity import CHAOS, compare, random_inputs
from test_oracle import random_reads

pytestmark = pytest.mark.gpu


def run_reads(cfg, ticks, seed, make_gpu=None):
    gpu = make_gpu() if make_gpu else make("gpu", **cfg)
    ora = make("c", **cfg)
    gpu.bootstrap()
    ora.bootstrap()
    rng = np.random.default_rng(seed)
    G, R = ora.G, ora.R
    ready = 0
    for t in range(ticks):
        reqs = random_reads(rng, G, R, t, p=0.2)
        gpu.read_index(reqs)
        assert ora.read_index(reqs) == 0
        ins = random_inputs(rng, G, R, cfg["max_entries_per_msg"])
        gpu.tick(*ins)
        ora.tick(*ins)
        compare(gpu, ora, t)
        got = gpu.read_ready_all()
        want = {r: ora.read_ready(r) for r in range(G * R)}
        want = {r: v for r, v in want.items() if v}
        assert got == want, t
        ready += sum(len(v) for v in want.values())
    assert ready > 0
    return ready


@pytest.mark.parametrize("R", [1, 2, 3, 5])
def test_read_index_chaos(R):
    cfg = dict(CHAOS, groups=4, replicas=R, payload_bytes=16, max_entries_per_msg=8, seed=600 + R)
    run_reads(cfg, ticks=120, seed=R)


def test_read_index_no_loss():
    """Without drops every follower's forwarded read comes back as a ReadIndexResp."""
    cfg = dict(CHAOS, groups=8, replicas=3, payload_bytes=16, max_entries_per_msg=8, drop_ppm=0, seed=17)
    assert run_reads(cfg, ticks=80, seed=11) > 30


@pytest.mark.parametrize("ranks", [2, 3])
def test_read_index_cluster(ranks):
    """Requests and ReadIndex/ReadIndexResp messages crossing ranks through the wire exchange."""
    from raftd_amd.cluster import LoopbackCluster
    cfg = dict(CHAOS, groups=2 * ranks, replicas=3, payload_bytes=16, max_entries_per_msg=8, seed=21 + ranks)
    run_reads(cfg, ticks=80, seed=ranks, make_gpu=lambda: LoopbackCluster(ranks=ranks, **cfg))


def test_read_index_survives_dropped_heartbeat():
    """The leader's read heartbeat is lost; the next regular heartbeat carries the pending ctx."""
    from test_oracle import read_heartbeat_drop
    cfg = dict(groups=1, replicas=3, payload_bytes=16, max_entries_per_msg=8, log_capacity=256, snapshot_entries=0,
               heartbeat_rtt=2, election_rtt=20)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    assert read_heartbeat_drop(gpu) == read_heartbeat_drop(ora)
    compare(gpu, ora, -1)


def test_read_index_errors():
    from raftd_amd.engine import RgError
    gpu = make("gpu", groups=2, replicas=3, payload_bytes=16)
    gpu.bootstrap()
    for bad in ([(2, 0, 1)], [(0, 3, 1)], [(0, 0, 0)]):
        with pytest.raises(RgError):
            gpu.read_index(bad)
    gpu.tick()
    assert gpu.read_ready_all() == {}


def test_read_index_queue():
    """dragonboat's readIndex queue on the device: four reads queue while the followers are cut off,
    a fifth is dropped, and one confirmation releases the four in arrival order at one index — as the
    oracle does (tests/test_oracle.py::read_queue)."""
    from test_oracle import read_queue
    cfg = dict(groups=1, replicas=3, payload_bytes=16, max_entries_per_msg=8, log_capacity=256, snapshot_entries=0,
               heartbeat_rtt=2, election_rtt=20)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    got = read_queue(gpu)
    assert got == read_queue(ora) and [c for c, _ in got[0]] == [100, 101, 102, 103]
    compare(gpu, ora, -1)
