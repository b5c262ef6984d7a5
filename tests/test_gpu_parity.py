"""GPU parity: the HIP engine (through the C-ABI) against the C oracle, tick by tick.

Bit-exact comparison of every replica's state, every emitted message (headers + inline entry
terms) and every log entry (term, type, len, CRC) on seeded random traces, plus payload bytes
and zlib CRCs at the end. 'Bit-exact' = with the restatement of DESIGN.md §1 (parity against
dragonboat itself is unpinned).
"""
import zlib

import numpy as np
import pytest

from engines import make

pytestmark = pytest.mark.gpu


def random_inputs(rng, G, R, emax, p_none=0.3, p_camp=0.02, p_iso=0.05):
    pt = rng.integers(0, R, G).astype(np.uint8)
    pt[rng.random(G) < p_none] = 0xFF
    pc = rng.integers(1, emax + 1, G).astype(np.uint32)
    camp = (rng.random(G * R) < p_camp).astype(np.uint8)
    iso = (rng.random(G * R) < p_iso).astype(np.uint8)
    return pt, pc, camp, iso


def compare(gpu, ora, t, check_entries=True):
    G, R = ora.G, ora.R
    gv = gpu.replicas()
    for rid in range(G * R):
        ov = ora.replica(rid)
        assert gv[rid] == ov, f"tick {t} rid {rid}: " + str({k: (gv[rid][k], ov[k]) for k in ov if gv[rid][k] != ov[k]})
        for d in range(R):
            gm, om = gpu.msgs(rid, d), ora.msgs(rid, d)
            assert gm == om, f"tick {t} msgs {rid}->{d}\n gpu {gm}\n ora {om}"
        if check_entries and ov["last"] > ov["marker"]:
            ge = gpu.entries(rid, ov["marker"] + 1, ov["last"] - ov["marker"])
            oe = [ora.entry(rid, i) for i in range(ov["marker"] + 1, ov["last"] + 1)]
            assert ge == oe, f"tick {t} entries rid {rid}"


def crc32c_py(b: bytes) -> int:
    """CRC-32C (Castagnoli, reflected 0x82F63B78), bit at a time: independent of both engines."""
    c = 0xFFFFFFFF
    for x in b:
        c ^= x
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
    return c ^ 0xFFFFFFFF


def check_payloads(gpu, ora, sample=4):
    G, R = ora.G, ora.R
    if not ora.cfg["payload_bytes"]:
        return
    for rid in range(0, G * R, max(1, G * R // sample)):
        v = ora.replica(rid)
        lo = max(v["marker"] + 1, v["last"] - 31)
        if v["last"] < lo:
            continue
        ge = gpu.entries(rid, lo, v["last"] - lo + 1, with_payload=True)
        for k, i in enumerate(range(lo, v["last"] + 1)):
            oe = ora.entry(rid, i, with_payload=True)
            assert ge[k]["payload"] == oe["payload"], (rid, i)
            want = crc32c_py(ge[k]["payload"]) if ora.cfg.get("crc32c") else zlib.crc32(ge[k]["payload"])
            assert ge[k]["crc"] == (want if ge[k]["len"] else 0)


def run_pair(cfg, ticks, seed, check_every=1, **inkw):
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    gpu.bootstrap()
    ora.bootstrap()
    compare(gpu, ora, -1)
    rng = np.random.default_rng(seed)
    for t in range(ticks):
        ins = random_inputs(rng, ora.G, ora.R, cfg.get("max_entries_per_msg", 64), **inkw)
        gpu.tick(*ins)
        ora.tick(*ins)
        if t % check_every == 0 or t == ticks - 1:
            compare(gpu, ora, t)
    check_payloads(gpu, ora)
    return gpu, ora


CHAOS = dict(log_capacity=64, payload_bytes=16, max_entries_per_msg=8, snapshot_entries=20,
             compaction_overhead=5, drop_ppm=150000)


@pytest.mark.parametrize("R", [1, 2, 3, 4, 5, 7])
def test_chaos_small(R):
    run_pair(dict(groups=4, replicas=R, seed=7 + R, **CHAOS), ticks=120, seed=R)


@pytest.mark.parametrize("P", [16, 256, 1024])
def test_chaos_crc32c(P):
    """rg_config.crc32c = 1: every entry CRC is CRC-32C, bit-exact with the oracle."""
    run_pair(dict(groups=6, replicas=3, seed=17, crc32c=1, **dict(CHAOS, payload_bytes=P)), ticks=100, seed=P,
             check_every=5)


@pytest.mark.parametrize("P", [0, 32, 64, 256, 1024])
def test_chaos_payload_sizes(P):
    cfg = dict(CHAOS, payload_bytes=P, max_entries_per_msg=16)
    run_pair(dict(groups=3, replicas=3, seed=99, **cfg), ticks=100, seed=P + 1)


def test_chaos_r5_heavy_loss():
    cfg = dict(CHAOS, drop_ppm=300000, max_msgs_per_pair=4)
    run_pair(dict(groups=6, replicas=5, seed=5, **cfg), ticks=200, seed=55, p_camp=0.05, p_iso=0.1)


def test_steady_state_c2_shape():
    """C2 shape at small scale: leaders elected on slot 0, 64-entry batches of 256 B every tick."""
    G, R = 64, 3
    cfg = dict(groups=G, replicas=R, log_capacity=2048, payload_bytes=256, max_entries_per_msg=64)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    for e in (gpu, ora):
        e.bootstrap()
        e.tick()
        camp = np.zeros(G * R, np.uint8)
        camp[0::R] = 1
        e.tick(campaign=camp)
    compare(gpu, ora, 1)
    pt, pc = np.zeros(G, np.uint8), np.full(G, 64, np.uint32)
    for t in range(40):
        gpu.tick(pt, pc)
        ora.tick(pt, pc)
        if t % 5 == 4:
            compare(gpu, ora, t, check_entries=(t % 20 == 19))
    check_payloads(gpu, ora, sample=8)
    v = gpu.replica(0)
    assert v["role"] == 2 and v["committed"] > 2000 and v["err"] == 0


def test_compaction_and_snapshot_path():
    """Small ring + frequent snapshots + isolation: exercises InstallSnapshot and restore."""
    cfg = dict(groups=4, replicas=3, log_capacity=32, payload_bytes=16, max_entries_per_msg=8,
               snapshot_entries=10, compaction_overhead=2, seed=3)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    gpu.bootstrap()
    ora.bootstrap()
    rng = np.random.default_rng(3)
    snaps = 0
    for t in range(150):
        pt = np.zeros(4, np.uint8)
        pc = rng.integers(1, 9, 4).astype(np.uint32)
        iso = np.zeros(12, np.uint8)
        if 20 <= t % 50 < 40:
            iso[2::3] = 1  # slot 2 partitioned for 20 ticks, then rejoins behind the compaction point
        camp = np.zeros(12, np.uint8)
        if t == 1:
            camp[0::3] = 1
        gpu.tick(pt, pc, camp, iso)
        ora.tick(pt, pc, camp, iso)
        compare(gpu, ora, t)
        for rid in range(12):
            snaps += sum(1 for m in ora.msgs(rid, 2) if m["type"] == 16)
    assert snaps > 0


def test_chaos_full_batches():
    """64-entry jobs under loss, elections and truncation: entries 32..63 of a job take their bank
    bits from the high half of the job's 64-bit masks (a sign-extending lane broadcast once set
    that half whenever entry 31's bit was set)."""
    cfg = dict(CHAOS, log_capacity=256, max_entries_per_msg=64, snapshot_entries=120, payload_bytes=16)
    run_pair(dict(groups=8, replicas=3, seed=31, **cfg), ticks=150, seed=64, p_camp=0.04)
