"""Cross-GPU replica placement against the oracle of the whole shard set.

N ranks run as N engines on one GPU (LoopbackCluster): replicas of a group live on different
ranks and every message between them goes through the wire (plan → pack → copy → unpack), with
followers reading entry payloads and sender CRCs out of the receive buffer. The single-process
C oracle steps all N * groups shards; every replica view, outbound message, log entry and payload
must be bit-identical. A two-process run drives the same exchange through torch.distributed.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from engines import make
from test_gpu_parity import CHAOS, check_payloads, compare, random_inputs

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def cluster_pair(ranks, cfg, wire_all=0):
    from raftd_amd.cluster import LoopbackCluster
    cl = LoopbackCluster(ranks=ranks, wire_all=wire_all, **cfg)
    ora = make("c", **cfg)
    cl.bootstrap()
    ora.bootstrap()
    return cl, ora


def run_chaos(ranks, cfg, ticks, seed, wire_all=0, **inkw):
    cl, ora = cluster_pair(ranks, cfg, wire_all)
    compare(cl, ora, -1)
    rng = np.random.default_rng(seed)
    for t in range(ticks):
        ins = random_inputs(rng, ora.G, ora.R, cfg.get("max_entries_per_msg", 64), **inkw)
        cl.tick(*ins)
        ora.tick(*ins)
        compare(cl, ora, t)
    check_payloads(cl, ora)
    return cl, ora


@pytest.mark.parametrize("ranks,R", [(2, 3), (3, 3), (4, 3), (8, 3), (8, 5), (4, 5), (2, 2), (2, 5), (3, 8)])
def test_cluster_chaos(ranks, R):
    cfg = dict(groups=2 * ranks, replicas=R, seed=11 + ranks + R, **CHAOS)
    run_chaos(ranks, cfg, ticks=100, seed=ranks * 10 + R)


def test_wire_all_one_rank():
    """One rank, every plane forced through the wire: the exchange alone must not change a bit."""
    cfg = dict(groups=6, replicas=3, seed=23, **CHAOS)
    run_chaos(1, cfg, ticks=100, seed=5, wire_all=1)


@pytest.mark.parametrize("P", [0, 1024])
def test_cluster_payload_sizes(P):
    cfg = dict(CHAOS, payload_bytes=P, max_entries_per_msg=16)
    run_chaos(4, dict(groups=8, replicas=3, seed=7, **cfg), ticks=60, seed=P + 3)


def test_cluster_steady_state_and_snapshots():
    """Config-3 shape at small scale (5 replicas on 8 ranks, 64-entry batches of 256 B), then a
    partition long enough for compaction to force InstallSnapshot across ranks."""
    G, R, N = 16, 5, 8
    cfg = dict(groups=G, replicas=R, log_capacity=256, payload_bytes=256, max_entries_per_msg=64,
               snapshot_entries=60, compaction_overhead=5, seed=9)
    cl, ora = cluster_pair(N, cfg)
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    for e in (cl, ora):
        e.tick()
        e.tick(campaign=camp)
    pt, pc = np.zeros(G, np.uint8), np.full(G, 64, np.uint32)
    snaps = 0
    for t in range(30):
        iso = np.zeros(G * R, np.uint8)
        if 8 <= t < 20:
            iso[4::R] = 1
        cl.tick(pt, pc, isolate=iso)
        ora.tick(pt, pc, isolate=iso)
        compare(cl, ora, t, check_entries=(t % 5 == 4))
        snaps += sum(1 for g in range(G) for m in ora.msgs(g * R, 4) if m["type"] == 16)
    check_payloads(cl, ora, sample=16)
    assert snaps > 0
    # the rejoining replica's higher term deposes some leaders (no PreVote, as raftd configures
    # dragonboat) — the oracle agrees bit for bit; every group still committed > 800 entries
    assert min(cl.replica(g * R)["committed"] for g in range(G)) > 800
    assert cl.wire_bytes > 0


def test_cluster_rejects_tick_without_exchange():
    from raftd_amd import RgError
    from raftd_amd.cluster import LoopbackCluster
    cl = LoopbackCluster(ranks=2, groups=4, replicas=3, log_capacity=64, payload_bytes=16,
                         max_entries_per_msg=8)
    cl.bootstrap()
    cl.tick()
    with pytest.raises(RgError, match="exchanged"):
        cl.engines[0].tick()


def test_two_processes_gloo():
    """Two processes on the one GPU, regions staged through host memory by gloo all_to_all."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
    out = subprocess.run([sys.executable, "-u", os.path.join(HERE, "dist_worker.py"), "2"], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "dist parity ok" in out.stdout


def test_two_processes_gloo_fixed_capacity():
    """The same two processes with the fixed-capacity sizing (rg_wire_plan_fixed: no host sync, no
    size exchange; the worst case of this configuration fits the first capacity, so nothing drops)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29543", DIST_FIXED="1")
    out = subprocess.run([sys.executable, "-u", os.path.join(HERE, "dist_worker.py"), "2"], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "dist parity ok" in out.stdout


def test_two_processes_capacities_agree_while_growing():
    """fixed-capacity regions that start at 4 KiB over two processes — units drop, both
    ends of every link grow its capacity from their own copy of the needs, and in every exchange the
    capacity a rank sends with equals the one its peer receives with; the drops stop and every
    shard's committed log is the same on all of its replicas (tests/capacity_worker.py)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29547")
    out = subprocess.run([sys.executable, "-u", os.path.join(HERE, "capacity_worker.py"), "2"], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "capacity agreement ok" in out.stdout


def test_cluster_full_batches():
    cfg = dict(CHAOS, log_capacity=256, max_entries_per_msg=64, snapshot_entries=120, payload_bytes=16)
    run_chaos(3, dict(groups=9, replicas=3, seed=37, **cfg), ticks=120, seed=65, p_camp=0.04)


def test_column_halves_match_oracle_windows():
    """A rank's columns split over two engines (column_base): each half cluster reproduces its
    window of the oracle of all groups — the layout DistEngine(halves=2) pipelines."""
    from raftd_amd.cluster import LoopbackCluster
    N, G, R = 4, 16, 3
    cfg = dict(replicas=R, seed=71, **CHAOS)
    halves = [LoopbackCluster(ranks=N, groups=G // 2, column_base=h * (G // 2) // N, **cfg) for h in range(2)]
    oras = [make("c", groups=G // 2, group_base=h * G // 2, **cfg) for h in range(2)]
    for x in halves + oras:
        x.bootstrap()
    rng = np.random.default_rng(72)
    for t in range(80):
        pt, pc, camp, iso = random_inputs(rng, G, R, CHAOS["max_entries_per_msg"])
        for h in range(2):
            g0, n = h * G // 2, G // 2
            ins = (pt[g0:g0 + n], pc[g0:g0 + n], camp[g0 * R:(g0 + n) * R], iso[g0 * R:(g0 + n) * R])
            halves[h].tick(*ins)
            oras[h].tick(*ins)
            compare(halves[h], oras[h], t)


def test_two_processes_gloo_halves():
    """DistEngine(halves=2) in two processes: plain ticks, then pipelined step_device ticks."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29534")
    out = subprocess.run([sys.executable, "-u", os.path.join(HERE, "dist_worker.py"), "2", "2"], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "dist parity ok" in out.stdout


@pytest.mark.parametrize("p2p_self", [0, 1])
def test_one_rank_nccl_wire_halves(p2p_self):
    """The RCCL path on the one GPU: a world-size-1 nccl group, every message through the wire,
    two column halves — plain ticks, then pipelined step_device ticks whose exchanges are
    asynchronous RCCL transfers waited on by the engine stream. p2p_self: the region to the rank
    itself goes through the grouped isend / irecv pieces the N > 1 exchange uses (instead of being
    packed in place), bit-exact with the oracle either way."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29535 + 40 * p2p_self), DIST_P2P_SELF=str(p2p_self))
    out = subprocess.run([sys.executable, "-u", os.path.join(HERE, "dist_worker.py"), "1", "2", "nccl"], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "dist parity ok" in out.stdout


def test_chunked_exchange_rccl():
    """all_to_all_bytes through RCCL in pieces of at most A2A_CHUNK bytes per region: exact for
    ragged, empty and 1.5 GB regions (a single RCCL call corrupted regions above 1 GiB); and
    p2p_regions' grouped isend / irecv pieces (DistEngine's N > 1 path) with the send region at its
    own offset in the shared exchange buffer."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29536")
    out = subprocess.run([sys.executable, "-u", os.path.join(HERE, "a2a_worker.py")], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "a2a chunks ok" in out.stdout



def test_malformed_exchange_data_is_dropped():
    """Exchange data comes from another process: a unit whose message count exceeds K, and a
    Replicate whose entry count exceeds E, must not make the receiver index outside its planes.
    unpack_kernel keeps the well-formed messages before them (the rest are lost, as dropped
    messages are), and Raft's retries bring every replica back to the same log."""
    import torch
    from raftd_amd.cluster import LoopbackCluster, plane_offset
    G, R, E, N, M_REPLICATE = 8, 3, 8, 2, 12
    cl = LoopbackCluster(ranks=N, groups=G, replicas=R, log_capacity=64, payload_bytes=16, max_entries_per_msg=E)
    cols = G // N

    def units(a, k):  # receive units of rank k from rank a: (s, d, j) planes a sends to k
        return sum(1 for j in range(cols) for s_ in range(R) for d in range(R)
                   if s_ != d and (a + plane_offset(s_, d, j, N)) % N == k)

    cl.bootstrap()
    cl.tick()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    cl.tick(campaign=camp)
    pt, pc = np.zeros(G, np.uint8), np.full(G, 4, np.uint32)
    for _ in range(6):
        cl.tick(pt, pc)
    hits = {"count": 0, "entries": 0}

    def regions(k, buf, rsizes):
        off = 0
        for a, n in enumerate(rsizes):
            if n:
                nu = units(a, k)
                yield off, n, nu, -(-nu * 8 // 256) * 256
            off += n

    def put_u64(buf, at, v):
        buf[at:at + 8].copy_(torch.from_numpy(np.array([v], np.uint64).view(np.uint8)).to(buf.device))

    # a region: [256-B header][unit table][data] (raftgpu_wire.hip)
    def bad_count(k, buf, rsizes):
        for off, n, nu, tb in regions(k, buf, rsizes):
            tab = buf[off + 256:off + 256 + 8 * nu].cpu().numpy().view(np.uint64)
            busy = [u for u in range(nu) if int(tab[u]) & 0xFF]
            if len(busy) >= 2:  # the first unit with messages claims 255, the next one's data lies at 2^54 B
                put_u64(buf, off + 256 + 8 * busy[0], (int(tab[busy[0]]) & ~0xFF) | 0xFF)
                put_u64(buf, off + 256 + 8 * busy[1], (1 << 58) | (int(tab[busy[1]]) & 0xFF))
                hits["count"] += 1

    def bad_entries(k, buf, rsizes):
        for off, n, nu, tb in regions(k, buf, rsizes):
            reg = buf[off:off + n].cpu().numpy()
            tab = reg[256:256 + 8 * nu].view(np.uint64)
            for u in range(nu):
                h = 256 + tb + (int(tab[u]) >> 8) * 16
                for _ in range(int(tab[u]) & 0xFF):  # walk the unit's messages
                    w0 = int(reg[h:h + 8].view(np.uint64)[0])
                    if w0 & 0xFF == M_REPLICATE and w0 >> 32:  # the first Replicate claims 2^20 entries
                        put_u64(buf, off + h, (w0 & 0xFFFFFFFF) | (1 << 52))
                        hits["entries"] += 1
                        return
                    h += 64 + (w0 >> 32 if w0 & 0xFF == M_REPLICATE else 0) * (16 + 16)

    cl.on_recv = bad_count
    cl.tick(pt, pc)
    cl.on_recv = bad_entries
    cl.tick(pt, pc)
    cl.on_recv = None
    assert hits["count"] > 0 and hits["entries"] > 0
    for _ in range(12):
        cl.tick(pt, pc)
    for _ in range(6):
        cl.tick()
    views = cl.replicas()
    assert not any(v["err"] for v in views)
    for g in range(G):
        lasts = {int(views[g * R + s]["last"]) for s in range(R)}
        commits = {int(views[g * R + s]["committed"]) for s in range(R)}
        assert len(lasts) == 1 and len(commits) == 1, (g, lasts, commits)


def _worker(args, port):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    out = subprocess.run([sys.executable, "-u", os.path.join(HERE, "dist_worker.py")] + args, env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "dist parity ok" in out.stdout


def test_two_processes_gloo_c_exchange():
    """rg_wire_exchange (the C-ABI exchange a Go host calls) with a host-staged transport over
    gloo: two processes, two column halves each on its own stream — plain ticks, then pipelined
    durable step_device ticks, every replica bit-exact against the oracle."""
    _worker(["2", "2", "gloo", "c"], 29537)


def test_one_rank_rccl_c_exchange():
    """rg_wire_exchange with the library's built-in RCCL transport (librccl loaded at run time,
    communicator from rg_rccl_unique_id / rg_rccl_open): one rank, every message through the
    wire, two halves on their own streams."""
    _worker(["1", "2", "nccl", "c"], 29538)


@pytest.mark.parametrize("self_path", ["copy", "rccl"])
def test_c_exchange_one_engine_vs_oracle(self_path, monkeypatch):
    """A bare engine (no torch.distributed) exchanging through the built-in RCCL transport at
    world size 1, every plane through the wire: chaos ticks bit-exact against the oracle. The region
    to the rank itself is a device copy, or (RAFTGPU_RCCL_SELF=rccl) a grouped RCCL send/receive."""
    from raftd_amd.engine import Engine, rccl_close, rccl_transport, rccl_unique_id
    monkeypatch.setenv("RAFTGPU_RCCL_SELF", self_path)
    cfg = dict(groups=16, replicas=3, seed=91, **CHAOS)
    eng = Engine(wire_all=1, **cfg)
    ora = make("c", **cfg)
    t = rccl_transport(rccl_unique_id(), 1, 0, 0)
    try:
        eng.bootstrap()
        ora.bootstrap()
        rng = np.random.default_rng(92)
        sent = 0
        for k in range(60):
            if k:
                sent += eng.wire_exchange(t)
            ins = random_inputs(rng, 16, 3, CHAOS["max_entries_per_msg"])
            eng.tick(*ins)
            ora.tick(*ins)
            compare(eng, ora, k)
        assert sent == 0  # one rank: its only region is its own
    finally:
        eng.sync()
        rccl_close(t)


def test_c_exchange_transport_failures_surface_as_errors():
    """A transport callback that fails (raises, or returns sizes that are not this rank's own)
    makes rg_wire_exchange fail with RG_EHIP / RG_EINVAL instead of unpacking anything."""
    from raftd_amd.engine import Engine, PyTransport, RgError
    cfg = dict(groups=8, replicas=3, seed=93, **CHAOS)
    eng = Engine(wire_all=1, **cfg)
    eng.bootstrap()
    eng.tick(*random_inputs(np.random.default_rng(94), 8, 3, CHAOS["max_entries_per_msg"]))

    def a2a_raises(*_):
        raise RuntimeError("link down")

    bad = PyTransport(lambda vals: list(vals), a2a_raises)
    bad.nranks = 1
    with pytest.raises(RgError, match="alltoallv failed"):
        eng.wire_exchange(bad.t)
    assert isinstance(bad.error, RuntimeError)
    eng.sync()
    # exact sizing (rg_config.wire_exact): a transport whose size exchange lies is refused
    ex = Engine(wire_all=1, wire_exact=1, **cfg)
    ex.bootstrap()
    ex.tick(*random_inputs(np.random.default_rng(94), 8, 3, CHAOS["max_entries_per_msg"]))
    liar = PyTransport(lambda vals: [v + 16 for v in vals], lambda *a: None)
    liar.nranks = 1
    with pytest.raises(RgError, match="another rank's sizes"):
        ex.wire_exchange(liar.t)
    ex.sync()


def _copy_transport(calls, moved=None):
    """A one-rank Python transport: alltoallv copies each send region (send + soff[r], ssize[r] bytes)
    to its receive region (after the engine stream, before returning); allgather records that it was
    called; `moved` collects the bytes each call was asked to move."""
    import torch
    from raftd_amd.cluster import _dev_bytes
    from raftd_amd.engine import PyTransport

    def a2a(send, soff, ssize, recv, roff, rsize, stream):
        torch.cuda.synchronize()
        assert list(ssize) == list(rsize)
        for r, n in enumerate(ssize):
            if n:
                _dev_bytes(recv + roff[r], n, "cuda").copy_(_dev_bytes(send + soff[r], n, "cuda"))
        if moved is not None:
            moved.append(sum(ssize))
        torch.cuda.synchronize()

    t = PyTransport(lambda vals: calls.append(list(vals)) or list(vals), a2a)
    t.nranks = 1
    return t


@pytest.mark.parametrize("sizing", ["fixed", "exact"])
def test_exchange_is_one_collective_with_fixed_capacity(sizing):
    """rg_wire_exchange with fixed-capacity regions (the default) moves them with one transport call
    per tick and never asks for the sizes (no allgather); with the default capacity (the worst case of
    this configuration fits) nothing is dropped and every tick equals the oracle. Exact sizing
    (rg_config.wire_exact) asks the transport for the sizes once per exchange."""
    from raftd_amd.engine import Engine
    cfg = dict(groups=16, replicas=3, seed=95, **CHAOS)
    eng = Engine(wire_all=1, wire_exact=int(sizing == "exact"), **cfg)
    ora = make("c", **cfg)
    calls, moved = [], []
    t = _copy_transport(calls, moved)
    eng.bootstrap()
    ora.bootstrap()
    rng = np.random.default_rng(96)
    for k in range(50):
        if k:
            eng.wire_exchange(t.t)
        ins = random_inputs(rng, 16, 3, CHAOS["max_entries_per_msg"])
        eng.tick(*ins)
        ora.tick(*ins)
        compare(eng, ora, k)
    assert t.error is None and eng.wire_dropped() == 0
    assert (calls == []) if sizing == "fixed" else len(calls) == 49
    # one rank: its only region is the one to itself, packed where the unpack reads it (rg_wire_pack_at),
    # so the transport is asked to move nothing
    assert len(moved) == 49 and set(moved) == {0}


def test_fixed_capacity_overflow_drops_units_and_grows():
    """Regions far too small for the traffic (RAFTGPU_WIRE_CAP0 = 4 KiB): the units past a region's
    end are dropped and counted, the capacity grows from the needs two exchanges later, the drops
    stop, and the cluster keeps committing with every replica's committed log equal to its leader's
    (message loss is safe in Raft). A shard whose campaigns lost their votes elects later (a
    split vote or two after the drops end: one shard elected at tick 37 of this seed), maybe another
    slot, which the proposals (all to slot 0) then miss."""
    import os
    from raftd_amd.engine import Engine
    G, R, E = 256, 3, 16
    os.environ["RAFTGPU_WIRE_CAP0"] = "4096"
    try:
        eng = Engine(wire_all=1, groups=G, replicas=R, log_capacity=256, payload_bytes=64, max_entries_per_msg=E,
                     snapshot_entries=0, seed=97)
        calls = []
        t = _copy_transport(calls)
        eng.bootstrap()
        camp = np.zeros(G * R, np.uint8)
        camp[0::R] = 1
        pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
        drops = []
        for k in range(60):
            if k:
                eng.wire_exchange(t.t)
            eng.tick(*((None, None, camp) if k == 1 else (pt, pc) if k >= 4 else ()))
            drops.append(eng.wire_dropped())
        eng.sync()
    finally:
        del os.environ["RAFTGPU_WIRE_CAP0"]
    assert drops[-1] > 0 and drops[-1] == drops[-20], drops  # dropped early, none in the last 20 ticks
    views = eng.replicas()
    done = 0
    led = []
    for g in range(G):
        vs = views[g * R:(g + 1) * R]
        c = min(v["committed"] for v in vs)
        lo = max(v["marker"] for v in vs) + 1
        if c >= lo:
            ref = [x["term"] for x in eng.entries(g * R, lo, c - lo + 1)]
            for s in range(1, R):
                assert [x["term"] for x in eng.entries(g * R + s, lo, c - lo + 1)] == ref, g
            done += 1
        assert any(v["role"] == 2 for v in vs), g  # every shard has a leader
        if vs[0]["role"] == 2:  # proposals go to slot 0
            led.append(max(v["committed"] for v in vs))
    assert done > G // 2
    assert np.mean(np.array(led) > 40) > 0.9, sorted(led)[:20]
    assert np.median([max(views[g * R + s]["committed"] for s in range(R)) for g in range(G)]) > 200


def test_fixed_capacity_keeps_a_floor_through_idle():
    """a large link (its worst case above 64 MiB) starts at the steady bound and shrinks while
    the load is low, but never below min(its start, 64 MiB). 50 idle exchanges (heartbeats only), then
    full 64-entry batches of 256-B Cmds (a ~36-MB burst): nothing is dropped and the batches commit."""
    from raftd_amd.engine import Engine
    G, R, E = 1024, 3, 64
    eng = Engine(wire_all=1, groups=G, replicas=R, log_capacity=512, payload_bytes=256, max_entries_per_msg=E,
                 seed=98)
    calls = []
    t = _copy_transport(calls)
    eng.bootstrap()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
    for k in range(60):  # bring-up, then idle
        if k:
            eng.wire_exchange(t.t)
        eng.tick(*((None, None, camp) if k == 1 else ()))
    c0 = eng.sum_committed()
    for k in range(8):  # the burst
        eng.wire_exchange(t.t)
        eng.tick(pt, pc)
    eng.sync()
    assert t.error is None and eng.wire_dropped() == 0
    assert eng.sum_committed() - c0 >= G * E * 5


@pytest.mark.parametrize("ranks", [3, 1])
def test_control_fast_path_covers_the_wire_steady_state(ranks):
    """Replicas spread over ranks (3: every follower on another rank than its leader; 1 with wire_all:
    every message through the wire): in steady state the followers' Replicates and the leaders'
    responses arrive over the wire, and no replica leaves the control fast path (unpack_kernel marks a
    Replicate whose entry records hold one application ring word, which the fast step appends as one
    uniform WIRE job) — every tick bit-exact with the oracle, entries and payloads included."""
    import ctypes as C
    from raftd_amd.cluster import LoopbackCluster
    G, R, E = 96, 3, 64
    cfg = dict(replicas=R, log_capacity=256, payload_bytes=256, max_entries_per_msg=E, snapshot_entries=100,
               compaction_overhead=5, seed=0x5EED)
    cl = LoopbackCluster(ranks=ranks, groups=G, **cfg, **(dict(wire_all=1) if ranks == 1 else {}))
    ora = make("c", groups=G, **cfg)
    fn = cl.engines[0].L.rg_debug_ctl_slow
    fn.argtypes, fn.restype = [C.c_void_p, C.POINTER(C.c_uint32)], C.c_int
    n = C.c_uint32()
    cl.bootstrap()
    ora.bootstrap()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
    slow = []
    for t in range(40):
        ins = (None, None, camp) if t == 1 else (pt, pc) if t >= 6 else ()
        cl.tick(*ins)
        ora.tick(*ins)
        tot = 0
        for e in cl.engines:
            assert fn(e.h, C.byref(n)) == 0
            tot += n.value
        slow.append(tot)
        compare(cl, ora, t)
    check_payloads(cl, ora)
    assert (cl.wire_bytes > 0 or ranks == 1) and ora.replica(0)["snap_index"] > 0  # 1 rank: regions to itself
    assert slow[1] > 0 and max(slow[12:]) == 0, slow
