"""Worker of test_gpu_cluster.test_two_processes_gloo: N processes (one rank each, gloo) step a
DistEngine on the same GPU; rank 0 compares every replica with the C oracle of all shards.
usage: python dist_worker.py N"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

G_LOCAL, R, TICKS = 6, 3, 60
CFG = dict(replicas=R, log_capacity=64, payload_bytes=32, max_entries_per_msg=8, snapshot_entries=20,
           compaction_overhead=5, drop_ppm=100000, seed=77)


def inputs(rng, G):
    pt = rng.integers(0, R, G).astype(np.uint8)
    pt[rng.random(G) < 0.3] = 0xFF
    pc = rng.integers(1, 9, G).astype(np.uint32)
    camp = (rng.random(G * R) < 0.02).astype(np.uint8)
    iso = (rng.random(G * R) < 0.05).astype(np.uint8)
    return pt, pc, camp, iso


def worker(rank, n):
    dist.init_process_group("gloo", rank=rank, world_size=n)
    from raftd_amd.cluster import DistEngine
    de = DistEngine(groups=G_LOCAL, device=0, **CFG)
    de.eng.bootstrap()
    G = G_LOCAL * n
    rng = np.random.default_rng(3)
    views = []
    for t in range(TICKS):
        de.tick(*inputs(rng, G))
        mine = {}
        for lr, v in enumerate(de.eng.replicas()):
            _, gr = de.eng.global_id(lr)
            lo = max(v["marker"] + 1, v["last"] - 7)
            ents = de.eng.entries(lr, lo, v["last"] - lo + 1, with_payload=True) if v["last"] >= lo else []
            mine[gr] = (v, [de.eng.msgs(lr, d) for d in range(R)], lo, ents)
        allv = [None] * n
        dist.all_gather_object(allv, mine)
        views.append({k: x for d in allv for k, x in d.items()})
    if rank == 0:
        from oracle.pyoracle import Oracle
        ora = Oracle(groups=G, **CFG)
        ora.bootstrap()
        rng = np.random.default_rng(3)
        for t in range(TICKS):
            ora.tick(*inputs(rng, G))
            for gr in range(G * R):
                v, ms, lo, ents = views[t][gr]
                ov = ora.replica(gr)
                assert v == ov, (t, gr, {k: (v[k], ov[k]) for k in ov if v[k] != ov[k]})
                assert ms == [ora.msgs(gr, d) for d in range(R)], (t, gr)
                oe = [ora.entry(gr, i, with_payload=True) for i in range(lo, v["last"] + 1)]
                assert ents == oe, (t, gr)
        print("dist parity ok", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    n = int(sys.argv[1])
    mp.spawn(worker, args=(n,), nprocs=n, join=True)
