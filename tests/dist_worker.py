"""Worker of test_gpu_cluster's two-process tests: N processes (one rank each, gloo) step a
DistEngine (1 or 2 column halves) on the same GPU — chaos ticks through tick(), then steady
proposal ticks through the pipelined step_device() when there are two halves; rank 0 compares
every replica with the C oracle of all shards.
usage: python dist_worker.py N [halves [backend [exchange]]]   (exchange: torch | c)

backend nccl (N = 1 only: RCCL will not put two ranks on one GPU): the one rank sends every
message through the wire (wire_all), so each exchange is a real RCCL all_to_all_single — the
asynchronous one with its work-handle wait in the pipelined steps.

exchange c: the library's rg_wire_exchange moves the regions (the C-ABI path a Go host uses):
through its built-in RCCL transport on nccl, through a host-staged Python transport on gloo."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

G_LOCAL, R, TICKS, STEADY = 6, 3, 60, 12
CFG = dict(replicas=R, log_capacity=64, payload_bytes=32, max_entries_per_msg=8, snapshot_entries=20,
           compaction_overhead=5, drop_ppm=100000, seed=77)


def inputs(rng, G):
    pt = rng.integers(0, R, G).astype(np.uint8)
    pt[rng.random(G) < 0.3] = 0xFF
    pc = rng.integers(1, 9, G).astype(np.uint32)
    camp = (rng.random(G * R) < 0.02).astype(np.uint8)
    iso = (rng.random(G * R) < 0.05).astype(np.uint8)
    return pt, pc, camp, iso


def snapshot(de):
    mine = {}
    for p in de.parts:
        e = p.eng
        for lr, v in enumerate(e.replicas()):
            _, gr = e.global_id(lr)
            lo = max(v["marker"] + 1, v["last"] - 7)
            ents = e.entries(lr, lo, v["last"] - lo + 1, with_payload=True) if v["last"] >= lo else []
            mine[gr] = (v, [e.msgs(lr, d) for d in range(R)], lo, ents)
    return mine


def worker(rank, n, halves, backend, exchange="torch"):
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=n, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=n)
    from raftd_amd.cluster import DistEngine
    extra = dict(wire_all=1) if n == 1 else {}
    fixed = {"1": True, "0": False}.get(os.environ.get("DIST_FIXED", ""))  # sizing mode (None: the default)
    p2p_self = os.environ.get("DIST_P2P_SELF") == "1"  # nccl, one rank: the region to self through p2p pieces
    de = DistEngine(groups=G_LOCAL * halves, halves=halves, device=0, exchange=exchange, fixed=fixed,
                    p2p_self=p2p_self, **CFG, **extra)
    if backend == "nccl":
        assert de.async_ok
    de.bootstrap()
    G = G_LOCAL * halves * n
    rng = np.random.default_rng(3)
    views = []
    for t in range(TICKS):
        de.tick(*inputs(rng, G))
        allv = [None] * n
        dist.all_gather_object(allv, snapshot(de))
        views.append({k: x for d in allv for k, x in d.items()})
    steady = []
    if halves > 1:  # pipelined: every half's exchange overlaps the other half's tick
        pt = np.zeros(G, np.uint8)
        pc = np.full(G, 5, np.uint32)
        dpt = torch.tensor(pt, device="cuda")
        dpc = torch.tensor(pc.astype(np.int32), device="cuda")
        # durable pipelined steps: each half's persistence feed is appended to its WAL (fsync) after
        # its tick and before its messages leave the rank (DistEngine.step_device's persist hook)
        import tempfile
        from raftd_amd.wal import WAL, replay
        tmp = tempfile.mkdtemp(prefix=f"rgwal{rank}_")
        wals = {id(p.eng): WAL(os.path.join(tmp, f"half{h}.wal")) for h, p in enumerate(de.parts)}
        de.drain()
        for p in de.parts:
            wals[id(p.eng)].append(0, *p.eng.persist_collect(full=True), CFG["payload_bytes"])
        steps = [0]

        def persist(e):
            wals[id(e)].append(steps[0] + 1, *e.persist_collect(), CFG["payload_bytes"])

        for k in range(STEADY):
            steps[0] = k
            de.step_device(dpt.data_ptr(), dpc.data_ptr(), persist=persist)
        de.drain()
        de.sync()
        for p in de.parts:  # the WAL holds every replica's hard state and log as the engine does
            logs = replay(wals[id(p.eng)].path, R)
            for lr, v in enumerate(p.eng.replicas()):
                s = logs[p.eng.global_id(lr)[1]].state
                assert (s["term"], s["vote"], s["commit"], s["last"], s["marker"]) == \
                    (v["term"], v["vote"], v["committed"], v["last"], v["marker"]), (rank, lr)
        allv = [None] * n
        dist.all_gather_object(allv, snapshot(de))
        steady = {k: x for d in allv for k, x in d.items()}
    if rank == 0:
        from oracle.pyoracle import Oracle
        ora = Oracle(groups=G, **CFG)
        ora.bootstrap()
        rng = np.random.default_rng(3)
        for t in range(TICKS):
            ora.tick(*inputs(rng, G))
            check(ora, views[t], G, t)
        if halves > 1:
            for _ in range(STEADY):
                ora.tick(np.zeros(G, np.uint8), np.full(G, 5, np.uint32))
            check(ora, steady, G, "steady")
        print("dist parity ok", flush=True)
    de.close()
    dist.barrier()
    dist.destroy_process_group()


def check(ora, snap, G, t):
    for gr in range(G * R):
        v, ms, lo, ents = snap[gr]
        ov = ora.replica(gr)
        assert v == ov, (t, gr, {k: (v[k], ov[k]) for k in ov if v[k] != ov[k]})
        assert ms == [ora.msgs(gr, d) for d in range(R)], (t, gr)
        oe = [ora.entry(gr, i, with_payload=True) for i in range(lo, v["last"] + 1)]
        assert ents == oe, (t, gr)


if __name__ == "__main__":
    n = int(sys.argv[1])
    halves = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    backend = sys.argv[3] if len(sys.argv) > 3 else "gloo"
    exchange = sys.argv[4] if len(sys.argv) > 4 else "torch"
    mp.spawn(worker, args=(n, halves, backend, exchange), nprocs=n, join=True)
