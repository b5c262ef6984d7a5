"""Probe: the 64K x 3 workload as K independent engines of G/K groups, each on its own HIP stream,
ticked back to back, so one engine's latency-bound control kernel can run beside another's bulk
kernel (groups are independent: no data is shared between the engines). Prints ms per tick of the
whole workload for K = 1 and K = the given counts, alternated.
usage: python scripts/halves_probe.py [--groups 65536] [--steps 20] [--ks 1,2,4]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def run(K, G, R, E, P, L, steps, warmup, torch):
    from raftd_amd import Engine
    from bench import bring_up
    engs, strs = [], []
    for k in range(K):
        s = torch.cuda.Stream()
        e = Engine(groups=G // K, seed=0x5EED + k, replicas=R, log_capacity=L, payload_bytes=P,
                   max_entries_per_msg=E, device=0)
        e.set_stream(s.cuda_stream)
        engs.append(e)
        strs.append(s)
    pts = []
    for e, s in zip(engs, strs):
        with torch.cuda.stream(s):
            bring_up(e, e.tick, G // K, R)
            pt = torch.zeros(G // K, dtype=torch.uint8, device="cuda")
            pc = torch.full((G // K,), E, dtype=torch.int32, device="cuda")
            pts.append((pt, pc))
    torch.cuda.synchronize()

    def step():
        for e, (pt, pc) in zip(engs, pts):
            e.tick_device(pt.data_ptr(), pc.data_ptr())

    for _ in range(warmup):
        step()
    for e in engs:
        e.sync()
    torch.cuda.synchronize()
    c0 = sum(e.sum_committed() for e in engs)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    for e in engs:
        e.sync()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    c1 = sum(e.sum_committed() for e in engs)
    errs = sum(int((e.replica_array()["err"] != 0).sum()) for e in engs)
    out = {"engines": K, "ms_per_step": el * 1e3 / steps, "group_steps_per_s": G * steps / el,
           "commits_per_step": (c1 - c0) / steps, "commits_expected": G * E, "errs": errs}
    for e in engs:
        e.close()
    del engs
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=65536)
    ap.add_argument("--replicas", type=int, default=3)
    ap.add_argument("--entries", type=int, default=64)
    ap.add_argument("--payload", type=int, default=256)
    ap.add_argument("--log-capacity", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--ks", default="1,2,4")
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    for rep in range(2):
        for K in [int(x) for x in a.ks.split(",")]:
            r = run(K, a.groups, a.replicas, a.entries, a.payload, a.log_capacity, a.steps, a.warmup, torch)
            r["rep"] = rep
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
