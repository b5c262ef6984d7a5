"""Engine robustness under a corrupt control parameter block.

The control kernel verifies a checksum over its parameter block before it dereferences anything; on
a mismatch it skips the tick and sets a sticky error. The pool and payload stages that follow it
must then not act on the skipped tick's stale rows (pool_kernel would free ~2^24 bogus pages,
bulk_kernel would replay tick t-2's jobs), and rg_sync must report RG_EINVARIANT."""
import ctypes as C

import numpy as np
import pytest

from engines import make

pytestmark = pytest.mark.gpu


def test_corrupt_parameter_block_is_reported_and_harmless():
    from raftd_amd.engine import RgError
    G, R, E = 64, 3, 8
    gpu = make("gpu", groups=G, replicas=R, log_capacity=256, payload_bytes=64, max_entries_per_msg=E,
               snapshot_entries=20, compaction_overhead=3, seed=0xC0)
    gpu.bootstrap()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
    gpu.tick()
    gpu.tick(campaign=camp)
    for _ in range(12):  # steady state with compaction: the stream pages turn over every tick
        gpu.tick(prop_target=pt, prop_count=pc)
    gpu.sync()
    before = gpu.pool_stats()
    assert not before["failed"]
    fn = gpu.L.rg_debug_corrupt_params
    fn.argtypes, fn.restype = [C.c_void_p, C.c_uint32], C.c_int
    assert fn(gpu.h, 1) == 0
    gpu.tick(prop_target=pt, prop_count=pc)  # its block fails the checksum
    with pytest.raises(RgError) as ei:
        gpu.sync()
    assert ei.value.code == -5  # RG_EINVARIANT
    after = gpu.pool_stats()
    assert not after["failed"]
    assert after["free"] == before["free"], (before, after)  # the pool stage did not run on stale rows
    for _ in range(3):  # the engine stays poisoned, and later ticks neither fault nor touch the pool
        gpu.tick(prop_target=pt, prop_count=pc)
    with pytest.raises(RgError):
        gpu.sync()
    assert gpu.pool_stats()["free"] == before["free"]


def test_parameter_blocks_are_copied_once_per_chunk_in_steady_state():
    """launch_control_slot copies a chunk of 32 parameter blocks at once, speculated for the next ticks
    with the same inputs, and a tick whose block differs copies its own. Steady ticks then issue one copy
    per 32 ticks; ticks whose inputs change (no proposals, a campaign) copy their own block. Every
    replica equals the oracle through both."""
    G, R, E = 96, 3, 8
    cfg = dict(groups=G, replicas=R, log_capacity=256, payload_bytes=64, max_entries_per_msg=E,
               snapshot_entries=40, compaction_overhead=3, seed=0xB10C)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    fn = gpu.L.rg_debug_param_copies
    fn.argtypes, fn.restype = [C.c_void_p, C.POINTER(C.c_uint64)], C.c_int
    n = C.c_uint64()

    def copies():
        assert fn(gpu.h, C.byref(n)) == 0
        return n.value

    for e in (gpu, ora):
        e.bootstrap()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
    for t in range(6):
        ins = dict(campaign=camp) if t == 1 else {}
        gpu.tick(**ins)
        ora.tick(**ins)
    c0 = copies()
    for t in range(6, 32):  # the chunk of ticks 0-31 was speculated without proposals: each copies its own
        gpu.tick(prop_target=pt, prop_count=pc)
        ora.tick(prop_target=pt, prop_count=pc)
    assert copies() - c0 == 26
    c0 = copies()
    for t in range(96):  # steady from a chunk's first tick: the same inputs every tick
        gpu.tick(prop_target=pt, prop_count=pc)
        ora.tick(prop_target=pt, prop_count=pc)
    steady = copies() - c0
    assert steady == 96 // 32, steady
    c1 = copies()
    for t in range(24):  # inputs change every other tick: each changed tick copies its own block
        ins = dict(prop_target=pt, prop_count=pc) if t % 2 else {}
        gpu.tick(**ins)
        ora.tick(**ins)
    assert copies() - c1 >= 10
    for rid in range(G * R):
        assert gpu.replica(rid) == ora.replica(rid), rid
    gpu.sync()


@pytest.mark.parametrize("fb", ["0", "1"])
def test_control_fast_path_covers_the_steady_state(fb, monkeypatch):
    """The benchmark's steady state (leaders with full batches every tick, snapshots and compaction)
    never leaves the control fast path (rg_debug_ctl_slow = 0 per tick after the election), an
    election does (the full step runs for the candidates: in control_slow_kernel, fb 0, or in the
    fast kernel's own launch, fb 1), and every replica equals the oracle."""
    monkeypatch.setenv("RAFTGPU_CTL_FB", fb)
    G, R, E = 512, 3, 64
    cfg = dict(groups=G, replicas=R, log_capacity=256, payload_bytes=256, max_entries_per_msg=E,
               snapshot_entries=100, compaction_overhead=5, seed=0x5EED)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    fn = gpu.L.rg_debug_ctl_slow
    fn.argtypes, fn.restype = [C.c_void_p, C.POINTER(C.c_uint32)], C.c_int
    n = C.c_uint32()
    for e in (gpu, ora):
        e.bootstrap()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
    slow = []
    for t in range(40):
        ins = dict(campaign=camp) if t == 1 else dict(prop_target=pt, prop_count=pc) if t >= 6 else {}
        gpu.tick(**ins)
        ora.tick(**ins)
        assert fn(gpu.h, C.byref(n)) == 0
        slow.append(n.value)
    for rid in range(G * R):
        assert gpu.replica(rid) == ora.replica(rid), rid
    assert ora.replica(0)["snap_index"] > 0
    assert slow[1] > 0 and max(slow[12:]) == 0, slow
