"""Worker of test_gpu_cluster's capacity-agreement test: two processes (gloo, one GPU)
step a DistEngine whose fixed-capacity regions start far too small (RAFTGPU_WIRE_CAP0 = 4 KiB), so
units drop and the links grow — on both ends, each from its own copy of the needs (the sender from
its plan, the receiver from the region headers). Every exchange records the capacities
rg_wire_plan_fixed hands out; rank 0 checks that the capacity rank a sends to rank b with equals the
one rank b receives from rank a with, in every exchange, that the drops stop, and that every shard's
committed log is the same on all of its replicas (message loss is safe in Raft).
usage: python capacity_worker.py N"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

G_LOCAL, R, E, TICKS = 64, 3, 16, 60


def worker(rank, n):
    os.environ["RAFTGPU_WIRE_CAP0"] = "4096"
    dist.init_process_group("gloo", rank=rank, world_size=n)
    from raftd_amd.cluster import DistEngine
    de = DistEngine(groups=G_LOCAL, halves=1, device=0, fixed=True, replicas=R, log_capacity=256, payload_bytes=64,
                    max_entries_per_msg=E, snapshot_entries=0, seed=97)
    e = de.parts[0].eng
    caps = []
    plan = e.wire_plan_fixed

    def recording_plan():
        s, r = plan()
        caps.append((list(s), list(r)))
        return s, r

    e.wire_plan_fixed = recording_plan
    de.bootstrap()
    G = G_LOCAL * n
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
    drops = []
    for k in range(TICKS):
        de.tick(*((None, None, camp) if k == 1 else (pt, pc) if k >= 4 else ()))
        drops.append(e.wire_dropped())
    de.sync()
    logs = {}
    for lr, v in enumerate(e.replicas()):
        g, _ = e.global_id(lr)
        lo = v["marker"] + 1
        terms = [x["term"] for x in e.entries(lr, lo, v["committed"] - lo + 1)] if v["committed"] >= lo else []
        logs.setdefault(int(g), []).append((lo, terms, v["role"]))
    allc, alld, alll = [None] * n, [None] * n, [None] * n
    dist.all_gather_object(allc, caps)
    dist.all_gather_object(alld, drops)
    dist.all_gather_object(alll, logs)
    if rank == 0:
        nx = len(allc[0])
        assert nx >= TICKS - 1 and all(len(c) == nx for c in allc), [len(c) for c in allc]
        grew = False
        for k in range(nx):
            for a in range(n):
                for b in range(n):
                    if a != b:
                        assert allc[a][k][0][b] == allc[b][k][1][a], (k, a, b, allc[a][k][0][b], allc[b][k][1][a])
                        grew |= allc[a][k][0][b] > allc[a][0][0][b]
        assert grew, "no capacity grew: the test did not exercise the adaptation"
        tot = [sum(d[k] for d in alld) for k in range(TICKS)]
        assert tot[-1] > 0 and tot[-1] == tot[-20], tot  # units dropped early, none in the last 20 ticks
        merged = {}
        for d in alll:
            for g, xs in d.items():
                merged.setdefault(g, []).extend(xs)
        agree = 0
        for g, xs in merged.items():
            assert len(xs) == R, (g, len(xs))
            lo = max(x[0] for x in xs)
            c = min(x[0] + len(x[1]) - 1 for x in xs)
            if c >= lo:
                ref = xs[0][1][lo - xs[0][0]:c - xs[0][0] + 1]
                for x in xs[1:]:
                    assert x[1][lo - x[0]:c - x[0] + 1] == ref, g
                agree += 1
            assert any(x[2] == 2 for x in xs), g  # every shard has a leader
        assert agree > len(merged) // 2, agree
        print(f"capacity agreement ok: {nx} exchanges, drops {tot[-1]}", flush=True)
    de.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    n = int(sys.argv[1])
    mp.spawn(worker, args=(n,), nprocs=n, join=True)
