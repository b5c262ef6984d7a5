"""Control-step time under an election storm (C4's shape: 65,536 x 3, random campaigns and isolation
every tick, so most replicas take the full step): mean control time per tick from HIP events, for
A/B of the full step's build (RAFTGPU_LIB)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from raftd_amd.engine import Engine  # noqa: E402

G, R = int(sys.argv[1]) if len(sys.argv) > 1 else 65536, 3
eng = Engine(groups=G, replicas=R, payload_bytes=256, max_entries_per_msg=64, log_capacity=2048, seed=0xC4)
eng.bootstrap()
rng = np.random.default_rng(4)
ins = [((rng.random(G * R) < 0.05).astype(np.uint8), (rng.random(G * R) < 0.05).astype(np.uint8)) for _ in range(8)]
for t in range(10):
    eng.tick(None, None, *ins[t % 8])
eng.sync()
eng.timing(True)
t0 = time.perf_counter()
for t in range(40):
    eng.tick(None, None, *ins[t % 8])
eng.sync()
wall = (time.perf_counter() - t0) * 1e3 / 40
print({"groups": G, "ms_per_tick": round(wall, 4), "kernel_ms_per_launch": {k: round(v[0] / max(v[1], 1), 4) for k, v in eng.kernel_ms().items()},
       "slow_lanes_note": "campaigns + isolation 5 % each per tick"}, flush=True)
