"""Probe: steady-state workload (slot-0 leaders, E-entry batches) on a direct engine and on a
wire_all engine (every message through plan/pack/unpack to itself) at G groups; compares
replica views every tick and reports the first divergence.
usage: wire_probe.py G [ticks] [payload] [log_capacity] [snapshot_entries]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from raftd_amd import Engine  # noqa: E402

G = int(sys.argv[1])
T = int(sys.argv[2]) if len(sys.argv) > 2 else 12
P = int(sys.argv[3]) if len(sys.argv) > 3 else 256
L = int(sys.argv[4]) if len(sys.argv) > 4 else 2048
SE = int(sys.argv[5]) if len(sys.argv) > 5 else 1000
R, E = 3, 64
cfg = dict(groups=G, replicas=R, log_capacity=L, payload_bytes=P, max_entries_per_msg=E, snapshot_entries=SE)
a = Engine(**cfg)
b = Engine(wire_all=1, **cfg)
buf = None


def xch():
    global buf
    sizes = b.wire_plan()
    n = sum(sizes)
    if buf is None or buf.numel() < n:
        buf = torch.empty(max(n, 1 << 20) * 3 // 2, dtype=torch.uint8, device="cuda")
    b.wire_pack(buf.data_ptr(), buf.numel())
    b.sync()
    b.wire_recv(buf.data_ptr(), sizes)
    b.sync()
    return n


for e in (a, b):
    e.bootstrap()
camp = np.zeros(G * R, np.uint8)
camp[0::R] = 1
pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
for t in range(T):
    ins = dict(campaign=camp) if t == 1 else (dict(prop_target=pt, prop_count=pc) if t >= 6 else {})
    a.tick(**ins)
    n = xch() if t > 0 else 0
    b.tick(**ins)
    b.sync()
    va, vb = a.replicas(), b.replicas()
    bad = [r for r in range(G * R) if va[r] != vb[r]]
    print(f"tick {t}: wire {n} B, diverged replicas {len(bad)}", flush=True)
    if bad:
        r = bad[0]
        print(r, {k: (va[r][k], vb[r][k]) for k in va[r] if va[r][k] != vb[r][k]})
        sys.exit(1)
print("probe ok", G)
