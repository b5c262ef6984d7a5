"""Randomised parity soak of the GPU engine against the C oracle (a GPU box run, not a test).

Each round draws a configuration — R 1..8, groups, payload size 0..256 (caller Cmds longer than P in
some rounds), ring and batch sizes, K, loss, snapshot / compaction settings, CRC polynomial, initial
membership — and runs it for a few hundred ticks with everything switched on at random: tick-input
proposal batches or caller Cmds (rg_propose), campaigns, isolation, membership changes, ReadIndex
requests. After every tick the replica views, every outbox message, the log window (term, type, len,
CRC) and the reads made ready must equal the oracle's; Cmd bytes are compared on sampled replicas.
Stops at the first mismatch and prints the round's seed and configuration.

usage: python scripts/soak.py [seconds] [first_seed] [ticks per configuration, default 200]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from engines import make  # noqa: E402
from test_gpu_parity import check_payloads, compare  # noqa: E402
from test_oracle import random_batches, random_ccs, random_reads  # noqa: E402


def draw(rng):
    R = int(rng.choice([1, 2, 3, 3, 4, 5, 5, 7, 8]))
    P = int(rng.choice([0, 16, 64, 256]))
    L = int(rng.choice([64, 128, 256]))
    E = int(rng.choice([4, 8, 16]))
    cfg = dict(groups=int(rng.integers(3, 24)), replicas=R, payload_bytes=P, log_capacity=L, max_entries_per_msg=E,
               max_msgs_per_pair=int(rng.choice([2, 4, 8])), snapshot_entries=int(rng.choice([0, 12, 20, 40])),
               compaction_overhead=int(rng.choice([2, 5])), drop_ppm=int(rng.choice([0, 20000, 100000, 200000])),
               heartbeat_rtt=int(rng.choice([1, 2])), election_rtt=int(rng.choice([10, 20])),
               crc32c=int(rng.integers(0, 2)), seed=int(rng.integers(1, 1 << 30)))
    if P and rng.random() < 0.3:
        cfg["max_cmd_bytes"] = int(rng.choice([P * 2, 1000, 5000]))
        cfg["pool_pages"] = cfg["groups"] * R * 64
    if R > 2 and rng.random() < 0.3:  # a partial initial membership (bit s = slot s)
        cfg["initial_members"] = int(rng.integers(1, 1 << R)) | 1
    return cfg


def run(seed, ticks):
    rng = np.random.default_rng(seed)
    cfg = draw(rng)
    # the engine under test: one engine (co-located planes), one engine with every message through the
    # wire (wire_all), or 2-4 engines as ranks of one cluster moving regions by device copies
    mode = str(rng.choice(["single", "wire_all", "ranks"], p=[0.45, 0.2, 0.35]))
    if os.environ.get("SOAK_KIND"):
        mode = "single"
    ranks = int(rng.integers(2, 5)) if mode == "ranks" else 1
    if mode == "ranks":
        cfg["groups"] = max(ranks, cfg["groups"] // ranks * ranks)
        if "pool_pages" in cfg:
            cfg["pool_pages"] = cfg["groups"] * cfg["replicas"] * 64
    if mode == "single":
        gpu = make(os.environ.get("SOAK_KIND", "gpu"), **cfg)
    else:
        from raftd_amd.cluster import LoopbackCluster
        gpu = LoopbackCluster(ranks=ranks, **dict(cfg, wire_all=1 if mode == "wire_all" else 0))
    ora = make("c", **cfg)
    G, R, E, P = cfg["groups"], cfg["replicas"], cfg["max_entries_per_msg"], cfg["payload_bytes"]
    gpu.bootstrap()
    ora.bootstrap()
    p_caller, p_cc, p_read = rng.choice([0.0, 0.5, 1.0]), rng.choice([0.0, 0.03]), rng.choice([0.0, 0.2])
    maxc = cfg.get("max_cmd_bytes")
    reads = 0
    for t in range(ticks):
        if p_cc and R > 1:
            for c in random_ccs(rng, G, R, p_cc):
                try:
                    ga = gpu.config_change(*c) or 0
                except Exception:  # RgError: refused (a change already staged for the group)
                    ga = -1
                assert (ga == 0) == (ora.config_change(*c) == 0), (seed, t, c)
        if p_read:
            rq = random_reads(rng, G, R, t, p=p_read)
            gpu.read_index(rq)
            ora.read_index(rq)
        camp = (rng.random(G * R) < 0.02).astype(np.uint8)
        iso = (rng.random(G * R) < 0.05).astype(np.uint8)
        if P and rng.random() < p_caller:
            batches = random_batches(rng, G, R, E, P, p_none=0.3, maxc=maxc)
            gpu.propose(batches)
            assert ora.propose(batches) == 0
            gpu.tick(None, None, camp, iso)
            ora.tick(None, None, camp, iso)
        else:
            pt = rng.integers(0, R, G).astype(np.uint8)
            pt[rng.random(G) < 0.3] = 0xFF
            pc = rng.integers(1, E + 1, G).astype(np.uint32)
            gpu.tick(pt, pc, camp, iso)
            ora.tick(pt, pc, camp, iso)
        try:
            compare(gpu, ora, t)
            got = gpu.read_ready_all()
            want = {r: v for r in range(G * R) if (v := ora.read_ready(r))}
            assert got == want, f"tick {t} reads\n gpu {got}\n ora {want}"
            reads += sum(len(v) for v in want.values())
            if t % 25 == 24:
                check_payloads(gpu, ora)
        except AssertionError as ex:
            print(f"MISMATCH seed {seed} mode {mode} ranks {ranks} cfg {cfg} p_caller {p_caller} p_cc {p_cc} p_read {p_read}\n{str(ex)[:3000]}",
                  flush=True)
            return False
    print(f"seed {seed} ok: {mode} x{ranks} G {G} R {R} P {P} L {cfg['log_capacity']} E {E} K {cfg['max_msgs_per_pair']} "
          f"drop {cfg['drop_ppm']} caller {p_caller} cc {p_cc} reads {reads} maxc {maxc} "
          f"members {cfg.get('initial_members', 0)}", flush=True)
    return True


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 300.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    ticks = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    t0, n = time.time(), 0
    while time.time() - t0 < budget:
        if not run(seed, ticks):
            sys.exit(1)
        seed += 1
        n += 1
    print(f"SOAK-OK {n} configurations in {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main()
