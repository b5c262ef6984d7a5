"""Debug helper: caller Cmds through one small engine; compares the log read path, the apply
copy-back and the oracle after every tick and prints the first mismatches."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from engines import make  # noqa: E402

cfg = dict(groups=1, replicas=int(sys.argv[1]) if len(sys.argv) > 1 else 1, payload_bytes=64,
           max_entries_per_msg=8, log_capacity=64)
gpu, ora = make("gpu", **cfg), make("c", **cfg)
for e in (gpu, ora):
    e.bootstrap()
    e.tick()
    e.tick(campaign=np.array([1] + [0] * (cfg["replicas"] - 1), np.uint8))
for _ in range(3):
    gpu.tick()
    ora.tick()
rng = np.random.default_rng(1)
for t in range(6):
    lens = [17, 29, 1, 64, 5, 40][t:] + [3]
    cmds = [((np.arange(n) + 16 * k + 100 * t) % 256).astype(np.uint8).tobytes() for k, n in enumerate(lens)]
    gpu.propose([(0, 0, cmds)])
    ora.propose([(0, 0, cmds)])
    gpu.tick()
    ora.tick()
    v = ora.replica(0)
    g = gpu.replica(0)
    print("tick", t, "last", v["last"], g["last"], "commit", v["committed"], g["committed"])
    for i in range(v["marker"] + 1, v["last"] + 1):
        oe = ora.entry(0, i, with_payload=True)
        ge = gpu.entry(0, i, with_payload=True)
        if oe != ge:
            print("  entry", i, "oracle", oe["len"], oe["crc"], oe["payload"][:20], "gpu", ge["len"], ge["crc"],
                  ge["payload"][:20])
    recs, packed = gpu.apply_committed_packed()
    want = ora.applied_entries(0)
    got = [(int(r["index"]), int(r["len"]), int(r["crc"]), bytes(packed[int(r["off"]):int(r["off"]) + int(r["len"])]))
           for r in recs if r["rid"] == 0]
    for a, b in zip(got, want):
        if a != b:
            print("  applied", a[:3], a[3][:20], "want", b[:3], b[3][:20])
    print("  applied offs", [(int(r["off"]), int(r["len"])) for r in recs if r["rid"] == 0], "packed", len(packed))
