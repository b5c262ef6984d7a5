"""Multi-rank host logic without a GPU: the placement math (Python vs the C++ of
raftgpu_internal.h through the host harness), its invariants, and the exchange transport over
torch.distributed with gloo at world_size 2."""
import ctypes as C
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from raftd_amd.cluster import (_offsets, all_to_all_bytes, exchange_sizes, global_group, local_rid, plane_offset,
                               rank_of)


@pytest.mark.parametrize("N", range(1, 17))
def test_placement_invariants(N):
    Gl = 24
    for R in range(1, 9):
        hosted = {}
        for g in range(N * Gl):
            ranks = [rank_of(g, s, N) for s in range(R)]
            if N >= R:
                assert len(set(ranks)) == R, (N, R, g, ranks)  # every replica on its own GPU
            for s, k in enumerate(ranks):
                j = local_rid(g, s, N, R) // R
                assert global_group(k, s, j, N) == g
                hosted.setdefault((k, s), set()).add(j)
        for k in range(N):
            for s in range(R):
                assert hosted[(k, s)] == set(range(Gl))  # each rank: one replica per (slot, column)


@pytest.mark.parametrize("N,R", [(8, 3), (8, 5), (4, 3), (16, 3), (7, 7)])
def test_leader_traffic_spreads_over_every_peer(N, R):
    """Over N - 1 consecutive columns a leader's followers sit at every other rank equally often,
    so no xGMI link carries more than (R - 1) / (N - 1) of a rank's leader→follower payload."""
    from collections import Counter
    cnt = Counter(plane_offset(0, d, j, N) for j in range(N - 1) for d in range(1, R))
    assert 0 not in cnt and set(cnt) == set(range(1, N)) and len(set(cnt.values())) == 1


@pytest.mark.parametrize("N,R", [(2, 3), (2, 5), (3, 5), (4, 5), (3, 8), (2, 8), (5, 8)])
def test_fewer_ranks_than_replicas_keeps_followers_home(N, R):
    """N < R: the leader's rank hosts ceil(R / N) replicas of each group (the fewest follower
    copies over xGMI), every rank at most that many, and the remote followers still spread over
    every peer evenly across N - 1 consecutive columns."""
    from collections import Counter
    hi = -(-R // N)
    for j in range(3 * (N - 1)):
        per_rank = Counter(plane_offset(0, d, j, N) for d in range(R))
        assert per_rank[0] == hi and max(per_rank.values()) == hi, (j, per_rank)
    cnt = Counter(plane_offset(0, d, j, N) for j in range(N - 1) for d in range(1, R))
    del cnt[0]
    assert set(cnt) == set(range(1, N)) and len(set(cnt.values())) == 1


def test_placement_matches_cpp():
    from native.ctl_host import build
    L = C.CDLL(build())
    L.ch_pl_group.restype = C.c_uint64
    L.ch_pl_group.argtypes = [C.c_uint32] * 4
    L.ch_pl_off.restype = C.c_uint32
    L.ch_pl_off.argtypes = [C.c_uint32] * 4
    for N in (1, 2, 3, 4, 5, 7, 8, 12, 16):
        for k in range(N):
            for s in range(8):
                for j in range(40):
                    assert L.ch_pl_group(N, k, s, j) == global_group(k, s, j, N)
        for s in range(8):
            for d in range(8):
                for j in range(20):
                    assert L.ch_pl_off(N, s, d, j) == plane_offset(s, d, j, N)


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _transport_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(100 + rank)
        sizes = [int(x) for x in torch.randint(0, 3000, (world,), generator=g)]
        sizes[rank] = 0 if rank == 0 else sizes[rank]  # an empty region and a self region
        offs, tot = _offsets(sizes)
        send = torch.empty(tot + 17, dtype=torch.uint8)
        for r in range(world):  # region r of rank a: bytes (a * 31 + r * 7 + i) mod 251
            i = torch.arange(sizes[r])
            send[offs[r]:offs[r] + sizes[r]] = ((rank * 31 + r * 7 + i) % 251).to(torch.uint8)
        rsizes, biggest = exchange_sizes(sizes)
        roffs, rtot = _offsets(rsizes)
        recv = torch.zeros(rtot + 5, dtype=torch.uint8)
        all_to_all_bytes(send, sizes, recv, rsizes)
        ok = True
        for a in range(world):
            i = torch.arange(rsizes[a])
            want = ((a * 31 + rank * 7 + i) % 251).to(torch.uint8)
            ok &= bool(torch.equal(recv[roffs[a]:roffs[a] + rsizes[a]], want))
        q.put((rank, ok and biggest >= max(sizes), rsizes))
    finally:
        dist.destroy_process_group()


def _p2p_worker(rank, world, port, q):
    """p2p_regions (the fixed-capacity exchange's transfer): every link's size is known to both of its
    ends without asking (here a formula of the pair), and regions move in pieces of at most 1,000 B."""
    from raftd_amd.cluster import p2p_regions
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        size = lambda a, b: 0 if (a + b) % 4 == 3 else (a * 997 + b * 613) % 2900 + 1  # noqa: E731
        sizes = [size(rank, r) for r in range(world)]
        rsizes = [size(a, rank) for a in range(world)]
        offs, tot = _offsets(sizes)
        send = torch.empty(tot + 9, dtype=torch.uint8)
        for r in range(world):
            i = torch.arange(sizes[r])
            send[offs[r]:offs[r] + sizes[r]] = ((rank * 31 + r * 7 + i) % 251).to(torch.uint8)
        roffs, rtot = _offsets(rsizes)
        recv = torch.zeros(rtot + 3, dtype=torch.uint8)
        p2p_regions(send, sizes, recv, rsizes, chunk=1000)
        ok = True
        for a in range(world):
            i = torch.arange(rsizes[a])
            want = ((a * 31 + rank * 7 + i) % 251).to(torch.uint8)
            ok &= bool(torch.equal(recv[roffs[a]:roffs[a] + rsizes[a]], want))
        q.put((rank, ok, rsizes))
    finally:
        dist.destroy_process_group()


def test_p2p_regions_gloo_world3():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_p2p_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res


def test_transport_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_transport_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res


@pytest.mark.parametrize("N,halves", [(1, 1), (2, 2), (3, 1), (8, 2)])
def test_dist_engine_routes_a_shard_to_its_half(N, halves):
    """DistEngine.propose / config_change / read_index route global shard g to half
    (g div N) div cols: the half whose columns hold g on the rank that hosts the replica."""
    cols = 12 // halves
    for rank in range(N):
        for h in range(halves):
            for s in range(3):
                for j in range(h * cols, (h + 1) * cols):
                    g = global_group(rank, s, j, N)
                    assert rank_of(g, s, N) == rank
                    assert (g // N) // cols == h
