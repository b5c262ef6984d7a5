"""The multi-tick path (rg_tick_device_n with RG_TICKN_GRAPH): k ticks captured as one
HIP graph and replayed must equal k rg_tick_device calls bit for bit — every replica view, every
outbox message and the newest log entries with payload — including ticks whose tick number matters
(deterministic message loss, randomized election timeouts) and snapshots / compaction. Both paths
are also checked against the C oracle directly after every block of ticks (not only
against single GPU ticks)."""
import numpy as np
import pytest
import torch

from engines import make
from test_gpu_parity import check_payloads, compare

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("payload", [0, 64])
def test_graph_ticks_equal_single_ticks(payload):
    G, R, K = 64, 3, 8
    cfg = dict(groups=G, replicas=R, log_capacity=256, payload_bytes=payload, max_entries_per_msg=16,
               snapshot_entries=40, compaction_overhead=5, drop_ppm=20000, seed=0x6A)
    a, b, ora = make("gpu", **cfg), make("gpu", **cfg), make("c", **cfg)
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    for e in (a, b, ora):
        e.bootstrap()
        e.tick()
        e.tick(campaign=camp)
        for _ in range(4):
            e.tick()
    pt_np = np.random.default_rng(3).integers(0, R, G).astype(np.uint8)
    pc_np = np.random.default_rng(4).integers(1, 17, G).astype(np.uint32)
    pt = torch.tensor(pt_np, dtype=torch.uint8, device="cuda")
    pc = torch.tensor(pc_np.astype(np.int32), dtype=torch.int32, device="cuda")
    for rep in range(5):
        for _ in range(K):
            a.tick_device(pt.data_ptr(), pc.data_ptr())
            ora.tick(pt_np, pc_np)
        b.tick_device_n(K, pt.data_ptr(), pc.data_ptr())
        a.sync()
        b.sync()
        assert a.t == b.t
        compare(b, ora, (rep + 1) * K)  # the graph path against the oracle itself
        check_payloads(b, ora)
        assert a.replica_array().tobytes() == b.replica_array().tobytes(), rep
        for rid in range(0, G * R, 7):
            for d in range(R):
                assert a.msgs(rid, d) == b.msgs(rid, d), (rep, rid, d)
            v = a.replica(rid)
            lo = max(v["marker"] + 1, v["last"] - 15)
            if v["last"] >= lo:
                assert a.entries(rid, lo, v["last"] - lo + 1, with_payload=True) == \
                    b.entries(rid, lo, v["last"] - lo + 1, with_payload=True), (rep, rid)
    v = b.replica_array()
    assert (v["err"] == 0).all() and v["snap_index"].max() > 0  # snapshots happened inside the graphs
    # a plain tick after the graphs continues the same run
    a.tick_device(pt.data_ptr(), pc.data_ptr())
    b.tick_device(pt.data_ptr(), pc.data_ptr())
    assert a.replica_array().tobytes() == b.replica_array().tobytes()


def test_graph_refuses_what_it_cannot_capture():
    from raftd_amd.engine import RgError
    e = make("gpu", groups=8, replicas=3, log_capacity=64, payload_bytes=16, max_entries_per_msg=4)
    e.bootstrap()
    with pytest.raises(RgError):
        e.tick_device_n(3)  # not a multiple of lcm(2, num_slabs)
    e.propose([(0, 0, [b"x"])])
    with pytest.raises(RgError):
        e.tick_device_n(2)  # a caller batch is staged


@pytest.mark.parametrize("R", [1, 3, 4])
def test_resident_ticks_equal_single_ticks(R):
    """RG_TICKN_RESIDENT (metadata-only engines): k ticks in one launch of the resident control kernel
    equal k rg_tick_device calls — elections from scratch inside the launch, message loss, isolation,
    snapshots and compaction; a group count that leaves the last workgroup partly empty."""
    G, K = 100, 16
    cfg = dict(groups=G, replicas=R, log_capacity=128, payload_bytes=0, max_entries_per_msg=16,
               snapshot_entries=30, compaction_overhead=4, drop_ppm=30000, seed=0x7E5 + R)
    a, b, ora = make("gpu", **cfg), make("gpu", **cfg), make("c", **cfg)
    for e in (a, b, ora):
        e.bootstrap()
    rng = np.random.default_rng(R)
    pt_np = rng.integers(0, R, G).astype(np.uint8)
    pc_np = rng.integers(1, 9, G).astype(np.uint32)
    iso_np = (rng.random(G * R) < 0.02).astype(np.uint8)
    pt = torch.tensor(pt_np, dtype=torch.uint8, device="cuda")
    pc = torch.tensor(pc_np.astype(np.int32), dtype=torch.int32, device="cuda")
    iso = torch.tensor(iso_np, device="cuda")
    for rep in range(6):
        for _ in range(K):
            a.tick_device(pt.data_ptr(), pc.data_ptr(), 0, iso.data_ptr())
            ora.tick(pt_np, pc_np, isolate=iso_np)
        b.tick_device_n(K, pt.data_ptr(), pc.data_ptr(), 0, iso.data_ptr(), resident=True)
        a.sync()
        b.sync()
        assert a.t == b.t
        compare(b, ora, (rep + 1) * K)  # the resident path against the oracle itself
        assert a.replica_array().tobytes() == b.replica_array().tobytes(), rep
        for rid in range(0, G * R, 11):
            for d in range(R):
                assert a.msgs(rid, d) == b.msgs(rid, d), (rep, rid, d)
    assert a.digest() == b.digest()
    v = b.replica_array()
    assert (v["role"] == 2).sum() > G // 2 and v["snap_index"].max() > 0  # elected, and snapshots ran


def test_resident_refuses_payload_engines():
    from raftd_amd.engine import RgError
    e = make("gpu", groups=8, replicas=3, log_capacity=64, payload_bytes=16, max_entries_per_msg=4)
    e.bootstrap()
    with pytest.raises(RgError):
        e.tick_device_n(4, resident=True)
