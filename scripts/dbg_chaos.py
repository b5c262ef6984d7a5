"""Debug helper: test_caller_cmds_chaos's run with per-tick entry checks; on the first mismatch,
prints the replica's window (len, CRCs, whether the bytes match) and the pool state."""
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from engines import make  # noqa: E402
from test_oracle import random_batches  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 1
P = int(sys.argv[2]) if len(sys.argv) > 2 else 64
cfg = dict(log_capacity=64, payload_bytes=P, max_entries_per_msg=8, snapshot_entries=20, compaction_overhead=5,
           drop_ppm=150000, groups=4, replicas=R, seed=40 + R)
gpu, ora = make("gpu", **cfg), make("c", **cfg)
gpu.bootstrap()
ora.bootstrap()
rng = np.random.default_rng(R * 100 + P)
G = 4
for t in range(100):
    batches = random_batches(rng, G, R, 8, P, p_none=0.3)
    gpu.propose(batches)
    assert ora.propose(batches) == 0
    camp = (rng.random(G * R) < 0.02).astype(np.uint8)
    iso = (rng.random(G * R) < 0.05).astype(np.uint8)
    gpu.tick(None, None, camp, iso)
    ora.tick(None, None, camp, iso)
    bad = None
    for rid in range(G * R):
        v = ora.replica(rid)
        gv = gpu.replica(rid)
        if v["last"] <= v["marker"]:
            continue
        ge = gpu.entries(rid, v["marker"] + 1, v["last"] - v["marker"], with_payload=True)
        oe = [ora.entry(rid, i, with_payload=True) for i in range(v["marker"] + 1, v["last"] + 1)]
        if ge != oe:
            bad = (rid, v, gv, ge, oe)
            break
    if bad:
        rid, v, gv, ge, oe = bad
        print("tick", t, "rid", rid, "marker", v["marker"], gv["marker"], "last", v["last"], gv["last"],
              "role", v["role"], "pool", gpu.pool_stats())
        for k, (a, b) in enumerate(zip(ge, oe)):
            i = v["marker"] + 1 + k
            flag = "" if a == b else "  <-- crc ok-for-bytes=%s bytes-equal=%s" % (
                a["crc"] == (zlib.crc32(a["payload"]) if a["len"] and a["type"] == 0 else 0), a["payload"] == b["payload"])
            print("  %3d t%d ty%d len %4d gcrc %08x ocrc %08x%s" % (i, a["term"], a["type"], a["len"], a["crc"], b["crc"],
                                                                  flag))
        print("batches this tick:", [(g, s, [len(c) for c in cm]) for g, s, cm in batches])
        break
else:
    print("no mismatch")
