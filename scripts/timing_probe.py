"""Why the bench's timed region (1.343 ms/tick) is slower than its untimed repeat (1.296 ms): three
timed blocks of 20 ticks back to back, then three untimed ones, each with and without the roofline's
bulk events, at the bench workload (64K x 3, 64 x 256-B entries per leader per tick)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from raftd_amd.engine import Engine  # noqa: E402

G, R, E, P = 65536, 3, 64, 256
eng = Engine(groups=G, replicas=R, payload_bytes=P, max_entries_per_msg=E, log_capacity=2048)
bench.bring_up(eng, eng.tick, G, R)
pt = torch.zeros(G, dtype=torch.uint8, device="cuda")
pc = torch.full((G,), E, dtype=torch.int32, device="cuda")


def block(n, events):
    eng.timing(events, bulk_only=True, every=4)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        eng.tick_device(pt.data_ptr(), pc.data_ptr())
    eng.sync()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / n
    eng.timing(False)
    return ms


for _ in range(5):
    eng.tick_device(pt.data_ptr(), pc.data_ptr())
for label, ev in (("events", True), ("none", False), ("events", True), ("none", False)):
    print(label, [round(block(20, ev), 4) for _ in range(3)], flush=True)
time.sleep(0.2)
print("after 0.2 s idle:", [round(block(20, False), 4) for _ in range(3)], flush=True)
