"""Client commands through the C-ABI (rg_propose) against the oracle (or_propose), tick by tick.

raftd hands every client command to the shard as an opaque `Cmd []byte`, and the state machine
gets it back verbatim as statemachine.Entry.Cmd (/root/reference/raft/state_machine.go:126-145).
Here variable-length Cmds (0, 1, 17 and payload_bytes bytes, and random lengths) enter through
rg_propose, are appended by leaders, forwarded by followers with their bytes, replicated, CRC'd over
exactly their length, compacted and copied back; every replica view, message, entry (term, type,
length, CRC, bytes) and applied batch must equal the oracle's. Parity with dragonboat itself is
unpinned.
"""
import zlib

import numpy as np
import pytest

from engines import make
from test_gpu_parity import CHAOS, compare, crc32c_py
from test_oracle import BIG_LENS, big_batches, random_batches

pytestmark = pytest.mark.gpu


def check_cmds(gpu, ora, crc32c=False):
    """Every log entry's bytes and CRC (the ring holds len bytes; the CRC covers exactly them)."""
    lens = set()
    for rid in range(ora.nrep):
        v = ora.replica(rid)
        if v["last"] <= v["marker"]:
            continue
        ge = gpu.entries(rid, v["marker"] + 1, v["last"] - v["marker"], with_payload=True)
        for k, i in enumerate(range(v["marker"] + 1, v["last"] + 1)):
            oe = ora.entry(rid, i, with_payload=True)
            assert ge[k] == oe, (rid, i)
            lens.add(oe["len"])
            want = crc32c_py(oe["payload"]) if crc32c else zlib.crc32(oe["payload"])
            assert ge[k]["crc"] == (want if oe["len"] else 0)
    return lens


def check_applied(gpu, ora):
    recs, pay = gpu.apply_committed()
    got = {}
    for r, p in zip(recs, pay):
        got.setdefault(int(r["rid"]), []).append((int(r["index"]), int(r["len"]), int(r["crc"]),
                                                  bytes(p[:int(r["len"])])))
    for rid in range(ora.nrep):
        assert got.get(rid, []) == ora.applied_entries(rid), rid


def run_caller(cfg, ticks, seed, make_gpu=None, check_every=1, p_none=0.3, applied=True, batches_fn=None):
    gpu = make_gpu() if make_gpu else make("gpu", **cfg)
    ora = make("c", **cfg)
    gpu.bootstrap()
    ora.bootstrap()
    rng = np.random.default_rng(seed)
    G, R, E, P = ora.G, ora.R, cfg["max_entries_per_msg"], cfg["payload_bytes"]
    for t in range(ticks):
        batches = (batches_fn(rng, G, R, P) if batches_fn else
                   random_batches(rng, G, R, E, P, p_none=p_none, maxc=cfg.get("max_cmd_bytes")))
        gpu.propose(batches)
        assert ora.propose(batches) == 0
        camp = (rng.random(G * R) < 0.02).astype(np.uint8)
        iso = (rng.random(G * R) < 0.05).astype(np.uint8)
        gpu.tick(None, None, camp, iso)
        ora.tick(None, None, camp, iso)
        if t % check_every == 0 or t == ticks - 1:
            compare(gpu, ora, t)
            if applied and hasattr(gpu, "apply_committed"):
                check_applied(gpu, ora)
    lens = check_cmds(gpu, ora, cfg.get("crc32c", 0))
    return gpu, ora, lens


@pytest.mark.parametrize("R,P", [(1, 64), (3, 16), (3, 256), (3, 1024), (5, 64), (4, 32)])
def test_caller_cmds_chaos(R, P):
    """Random-length Cmds under message loss, isolation, elections, truncation and snapshots."""
    cfg = dict(CHAOS, groups=4, replicas=R, payload_bytes=P, max_entries_per_msg=8, seed=40 + R)
    _, _, lens = run_caller(cfg, ticks=100, seed=R * 100 + P)
    assert {0, 1, P} <= lens and len(lens) > 4, lens


@pytest.mark.parametrize("R,P,maxc,pages", [(3, 64, 1000, 0), (5, 16, 300, 0), (3, 256, 8191, 0), (3, 64, 2000, 16),
                                            (1, 1024, 4096, 0), (4, 32, 700, 0)])
def test_caller_long_cmds_chaos(R, P, maxc, pages):
    """Cmds longer than payload_bytes (P - 1, P + 1, max_cmd_bytes, random up to it) through the paged
    payload stream: appended, forwarded, replicated, CRC'd, compacted (pages freed and reused) and
    copied back bit-exact with the oracle; pages = 16: the stream capacity rule refuses appends."""
    # a pool of stream_pages per replica never runs dry (the stream rule bounds live + pending pages);
    # the default pool (a full log of P-byte Cmds per replica) is sized for the benchmark's Cmds
    cfg = dict(CHAOS, groups=4, replicas=R, payload_bytes=P, max_entries_per_msg=8, seed=60 + R,
               max_cmd_bytes=maxc, stream_pages=pages, pool_pages=4 * R * (pages or 16))
    gpu, _, lens = run_caller(cfg, ticks=100, seed=R * 1000 + maxc)
    assert max(lens) > P and {0, 1} <= lens, lens
    st = gpu.pool_stats()
    assert not st["failed"] and 0 < st["free"] < st["total"], st


@pytest.mark.parametrize("R,P", [(3, 64), (3, 256), (5, 16)])
def test_caller_megabyte_cmds_chaos(R, P):
    """Cmds of 8,191, 8,192, 65,536 and 1 MiB bytes (max_cmd_bytes 1 MiB; r03 refused anything past
    8,191 B): under message loss, isolation, elections, truncation and snapshots every replica,
    message, entry (bytes and CRC) and applied batch equals the oracle's, tick by tick."""
    cfg = dict(CHAOS, groups=4, replicas=R, payload_bytes=P, max_entries_per_msg=8, seed=90 + R,
               max_cmd_bytes=1 << 20, pool_pages=4 * R * 2048)
    gpu, _, lens = run_caller(cfg, ticks=60, seed=R * 77 + P, batches_fn=big_batches)
    assert set(BIG_LENS) <= lens, lens
    st = gpu.pool_stats()
    assert not st["failed"], st


def test_caller_megabyte_cmds_cluster():
    """1-MiB Cmds over the wire: forwarded Proposes and Replicates carry them between ranks."""
    from raftd_amd.cluster import LoopbackCluster
    cfg = dict(CHAOS, groups=4, replicas=3, payload_bytes=64, max_entries_per_msg=8, seed=17,
               max_cmd_bytes=1 << 20, pool_pages=2 * 3 * 2048)
    _, _, lens = run_caller(cfg, ticks=50, seed=5, batches_fn=big_batches,
                            make_gpu=lambda: LoopbackCluster(ranks=2, **cfg))
    assert max(lens) == 1 << 20, lens


def test_caller_long_cmds_crc32c():
    cfg = dict(CHAOS, groups=4, replicas=3, payload_bytes=64, max_entries_per_msg=8, seed=6, crc32c=1,
               max_cmd_bytes=900, pool_pages=4 * 3 * 16)
    run_caller(cfg, ticks=80, seed=78)


@pytest.mark.parametrize("ranks,R", [(2, 3), (3, 5)])
def test_caller_long_cmds_cluster(ranks, R):
    """Long Cmds over the wire: a forwarded Propose and Replicate carry packed Cmds of any length."""
    from raftd_amd.cluster import LoopbackCluster
    cfg = dict(CHAOS, groups=2 * ranks, replicas=R, payload_bytes=64, max_entries_per_msg=8, seed=9 + ranks,
               max_cmd_bytes=1500, pool_pages=2 * ranks * R * 16)
    run_caller(cfg, ticks=80, seed=ranks * 11 + R, make_gpu=lambda: LoopbackCluster(ranks=ranks, **cfg))


def test_pool_exhaustion_poisons_the_engine():
    """A pool too small for the Cmds: the replicas whose pages could not be taken get RG_ERR_POOL
    (sticky), rg_pool_stats reports the failure, and nothing is written out of bounds."""
    from raftd_amd.engine import RG_ERR_POOL
    cfg = dict(groups=4, replicas=3, payload_bytes=64, max_entries_per_msg=8, log_capacity=64, max_cmd_bytes=4000,
               pool_pages=24)
    gpu = make("gpu", **cfg)
    gpu.bootstrap()
    camp = np.zeros(12, np.uint8)
    camp[0::3] = 1
    gpu.tick()
    gpu.tick(campaign=camp)
    for _ in range(3):
        gpu.tick()
    big = bytes(range(256)) * 15
    for t in range(6):
        gpu.propose([(g, 0, [big] * 8) for g in range(4)])
        gpu.tick()
    st = gpu.pool_stats()
    errs = [gpu.replica(r)["err"] for r in range(12)]
    assert st["failed"] and any(e & RG_ERR_POOL for e in errs), (st, errs)


def test_caller_cmds_crc32c():
    cfg = dict(CHAOS, groups=4, replicas=3, payload_bytes=256, max_entries_per_msg=8, seed=5, crc32c=1)
    run_caller(cfg, ticks=80, seed=77)


def test_caller_cmds_full_batches():
    """64-Cmd batches: the upper half of the jobs' 64-bit masks, all lengths in one batch."""
    cfg = dict(CHAOS, groups=4, replicas=3, payload_bytes=64, max_entries_per_msg=64, log_capacity=512,
               snapshot_entries=200, seed=8)
    run_caller(cfg, ticks=60, seed=64, check_every=3)


@pytest.mark.parametrize("ranks,R", [(2, 3), (3, 3), (4, 5), (2, 5)])
def test_caller_cmds_cluster(ranks, R):
    """Replicas on different ranks: a follower's forwarded proposal carries its Cmds over the wire
    to a leader on another rank (pack reads them from the forwarder's slab row)."""
    from raftd_amd.cluster import LoopbackCluster
    cfg = dict(CHAOS, groups=2 * ranks, replicas=R, payload_bytes=64, max_entries_per_msg=8, seed=3 + ranks)
    run_caller(cfg, ticks=80, seed=ranks * 7 + R, make_gpu=lambda: LoopbackCluster(ranks=ranks, **cfg))


def test_caller_cmds_metadata_only():
    """payload_bytes 0: every Cmd is empty; proposals still commit (no payload stage)."""
    cfg = dict(CHAOS, groups=4, replicas=3, payload_bytes=0, max_entries_per_msg=8, seed=2)
    from engines import make as mk
    gpu, ora = mk("gpu", **cfg), mk("c", **cfg)
    gpu.bootstrap()
    ora.bootstrap()
    rng = np.random.default_rng(1)
    for t in range(60):
        b = [(g, int(rng.integers(0, 3)), [b""] * int(rng.integers(1, 9))) for g in range(4)]
        gpu.propose(b)
        assert ora.propose(b) == 0
        gpu.tick()
        ora.tick()
        compare(gpu, ora, t)


def test_propose_errors_stage_nothing():
    from raftd_amd.engine import RG_EFULL, RG_EINVAL, RgError
    cfg = dict(groups=2, replicas=3, payload_bytes=16, max_entries_per_msg=4, log_capacity=64)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    for e in (gpu, ora):
        e.bootstrap()
    gpu.propose([(0, 1, [b"a"] * 3)])
    assert ora.propose([(0, 1, [b"a"] * 3)]) == 0
    cases = [([(0, 1, [b"b"] * 2)], RG_EFULL), ([(0, 2, [b"c"])], RG_EFULL), ([(1, 0, [b"b"] * 5)], RG_EINVAL),
             ([(0, 1, [b"x" * 17])], RG_EINVAL), ([(2, 0, [b"x"])], RG_EINVAL),
             ([(1, 0, [])], RG_EINVAL), ([(1, 0, [b"ok"]), (1, 2, [b"no"])], RG_EFULL)]
    for batch, code in cases:
        with pytest.raises(RgError) as ei:
            gpu.propose(batch)
        assert ei.value.code == code, batch
        assert ora.propose(batch) == code
    gpu.propose([(0, 1, [b""])])  # 4 = E
    assert ora.propose([(0, 1, [b""])]) == 0
    with pytest.raises(RgError):
        gpu.tick(np.zeros(2, np.uint8), np.ones(2, np.uint32))  # staged + tick-input proposals
    for e in (gpu, ora):
        e.tick()
    compare(gpu, ora, 0)


def test_caller_then_synthetic():
    """A synthetic (tick-input) proposal after caller proposals regenerates the slab bytes first."""
    cfg = dict(groups=4, replicas=3, payload_bytes=64, max_entries_per_msg=8, log_capacity=256)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    camp = np.zeros(12, np.uint8)
    camp[0::3] = 1
    for e in (gpu, ora):
        e.bootstrap()
        e.tick()
        e.tick(campaign=camp)
    rng = np.random.default_rng(9)
    for t in range(12):
        if t % 3 == 2:
            ins = (np.zeros(4, np.uint8), np.full(4, 8, np.uint32))
            gpu.tick(*ins)
            ora.tick(*ins)
        else:
            b = random_batches(rng, 4, 3, 8, 64, p_none=0.0)
            gpu.propose(b)
            ora.propose(b)
            gpu.tick()
            ora.tick()
        compare(gpu, ora, t)
    check_cmds(gpu, ora)


def _registered(gpu, cap):
    """gpu.propose through a buffer registered once (rg_host_register): rg_propose moves a call's Cmds
    by DMA straight from it when the packing allows, else through pinned staging."""
    from raftd_amd.engine import pack_proposals
    buf = np.zeros(cap, np.uint8)
    gpu.host_register(buf.ctypes.data, cap)

    def propose(batches):
        props, lens, blob = pack_proposals(batches)
        assert blob.size <= cap
        buf[:blob.size] = blob
        gpu._check(gpu.L.rg_propose(gpu.h, props, len(batches), buf.ctypes.data if blob.size else None,
                                    lens.ctypes.data if lens.size else None))
    return propose, buf


@pytest.mark.parametrize("R,P", [(3, 64), (3, 256), (5, 16)])
def test_caller_cmds_registered_buffer(R, P):
    """Cmds staged from a registered host buffer: ticks whose Cmds are all multiples of 16 B go by DMA
    straight from it (one run per call), the others (odd lengths inside a batch) through staging;
    either way every replica, entry (bytes, CRC) and applied batch equals the oracle's."""
    cfg = dict(CHAOS, groups=4, replicas=R, payload_bytes=P, max_entries_per_msg=8, seed=70 + R,
               max_cmd_bytes=4 * P)
    holder = {}

    def make_gpu():
        g = make("gpu", **cfg)
        holder["p"], holder["buf"] = _registered(g, 1 << 20)
        g.propose = holder["p"]
        return g

    def batches_fn(rng, G, R_, P_):
        aligned = rng.random() < 0.6
        out = []
        for g in range(G):
            if rng.random() < 0.3:
                continue
            n = int(rng.integers(1, 9))
            if aligned:
                cmds = [rng.integers(0, 256, 16 * int(rng.integers(0, 3 * P_ // 16 + 2)), dtype=np.uint8).tobytes()
                        for _ in range(n)]
            else:
                cmds = [rng.integers(0, 256, int(rng.integers(0, 2 * P_ + 3)), dtype=np.uint8).tobytes()
                        for _ in range(n)]
            out.append((g, int(rng.integers(0, R_)), cmds))
        return out

    gpu, _, lens = run_caller(cfg, ticks=60, seed=R * 31 + P, make_gpu=make_gpu, batches_fn=batches_fn)
    assert any(x % 16 for x in lens) and any(x and x % 16 == 0 for x in lens), lens
    gpu.host_unregister(holder["buf"].ctypes.data)


def test_large_call_staged_in_pieces_and_registered():
    """A call of 8,192 shards x 64 Cmds of 272 B (about 143 MB: three staged pieces, threaded batch
    scan) and the same from a registered buffer with some 7-B Cmds mixed in: the whole table equals the
    oracle's (rg_digest)."""
    from raftd_amd.engine import Proposal
    G, R, E, P = 8192, 3, 64, 256
    cfg = dict(groups=G, replicas=R, log_capacity=256, payload_bytes=P, max_entries_per_msg=E, snapshot_entries=0,
               max_cmd_bytes=512, seed=0x1A6E)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    for e in (gpu, ora):
        e.bootstrap()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    for e in (gpu, ora):
        e.tick()
        e.tick(campaign=camp)
        e.tick()
    rng = np.random.default_rng(5)
    buf = np.zeros(G * E * 272, np.uint8)
    gpu.host_register(buf.ctypes.data, buf.nbytes)
    try:
        for t in range(4):
            lens = np.full(G * E, 272, np.uint32)
            if t >= 2:  # odd lengths: staging; and the last Cmd of some batches odd: direct with more runs
                lens[rng.integers(0, G * E, 50)] = 7
                lens[np.arange(G) * E + E - 1] = 9 if t == 3 else 272
            blob = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
            props = (Proposal * G)()
            a = np.frombuffer(props, dtype=np.dtype([("group", "<u8"), ("slot", "<u4"), ("count", "<u4"),
                                                     ("first", "<u8")]))
            a["group"], a["slot"], a["count"] = np.arange(G), 0, E
            a["first"] = np.arange(G, dtype=np.uint64) * E
            src = buf if t % 2 else blob
            if t % 2:
                buf[:blob.size] = blob
            gpu._check(gpu.L.rg_propose(gpu.h, props, G, src.ctypes.data, lens.ctypes.data))
            cmds = np.split(blob, np.cumsum(lens)[:-1].astype(np.int64))
            batches = [(g, 0, [c.tobytes() for c in cmds[g * E:(g + 1) * E]]) for g in range(G)]
            assert ora.propose(batches) == 0
            gpu.tick()
            ora.tick()
            assert gpu.digest() == ora.digest(), t
    finally:
        gpu.host_unregister(buf.ctypes.data)
