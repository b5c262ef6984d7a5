"""Health of the one-rank RCCL rehearsal (bench --placement spread --wire-all) per tick: leaders,
commit sum and error bits of every replica, for a given size / halves / exchange mode.
usage: python scripts/rehearse_probe.py GROUPS HALVES {plain|pipelined} [entries payload]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29571")
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

G, H, mode = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
E = int(sys.argv[4]) if len(sys.argv) > 4 else 64
P = int(sys.argv[5]) if len(sys.argv) > 5 else 256
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
from raftd_amd.cluster import DistEngine  # noqa: E402

de = DistEngine(groups=G, halves=H, seed=0x5EED, wire_all=1, replicas=3, log_capacity=2048, payload_bytes=P,
                max_entries_per_msg=E, device=0)
R = 3


def health(tag):
    de.drain()
    de.sync()
    lead = com = 0
    errs = {}
    for p in de.parts:
        a = p.eng.replica_array()
        lead += int((a["role"] == 2).sum())
        com += int(a["committed"].sum())
        for b in np.unique(a["err"]):
            if b:
                errs[int(b)] = errs.get(int(b), 0) + int((a["err"] == b).sum())
    print(f"{tag}: leaders {lead}/{G} committed_sum {com} errors {errs}", flush=True)


de.bootstrap()
de.tick()
camp = np.zeros(G * R, np.uint8)
camp[0::R] = 1
de.tick(campaign=camp)
for t in range(4):
    de.tick()
health("after election")
pt = torch.zeros(G, dtype=torch.uint8, device="cuda")
pc = torch.full((G,), E, dtype=torch.int32, device="cuda")
for t in range(6):
    if mode == "pipelined":
        de.step_device(pt.data_ptr(), pc.data_ptr())
    else:
        de.tick_device(pt.data_ptr(), pc.data_ptr())
    health(f"{mode} tick {t}")
dist.destroy_process_group()
