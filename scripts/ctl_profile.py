"""Where control_kernel's time goes: phase stamps of an RG_CTL_PROFILE build at 64K x 3 steady
state (every leader proposes 64 entries per tick).
usage: python scripts/ctl_profile.py build_variants/ctlprof.so [groups [payload_bytes]]"""
import ctypes as C
import os
import sys

os.environ["RAFTGPU_LIB"] = os.path.abspath(sys.argv[1])
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from raftd_amd.engine import Engine  # noqa: E402

G, R, E = int(sys.argv[2]) if len(sys.argv) > 2 else 65536, 3, 64
P = int(sys.argv[3]) if len(sys.argv) > 3 else 256
eng = Engine(groups=G, replicas=R, log_capacity=2048, payload_bytes=P, max_entries_per_msg=E)
eng.bootstrap()
eng.tick()
camp = np.zeros(G * R, np.uint8)
camp[0::R] = 1
eng.tick(campaign=camp)
pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
for _ in range(12):
    eng.tick(pt, pc)
prof = np.zeros((12, G * R), np.uint32)
fn = eng.L.rg_debug_ctl_profile
fn.argtypes = [C.c_void_p, C.c_void_p]
assert fn(eng.h, prof.ctypes.data) == 0
d = (np.diff(prof[:6].astype(np.int64), axis=0) % 2**32).astype(np.float64)
acc = prof[6:].astype(np.float64)
accn = ["propose:append", "propose:broadcast", "handle_replicate", "write_entries", "-", "handle (all msgs)"]
names = ["load+inbox", "campaign+tick", "propose", "apply/snap", "store"]
roles = np.array([v for v in eng.replica_array()["role"]])
for s in range(R):
    sl = slice(s * G, (s + 1) * G)
    tot = d[:, sl].sum(axis=0)
    print(f"slot {s} (role {np.bincount(roles[s::R], minlength=3).tolist()} F/C/L): total {tot.mean():8.0f} cyc "
          f"(p50 {np.median(tot):.0f}, p99 {np.percentile(tot, 99):.0f})  " +
          "  ".join(f"{n} {d[k, sl].mean():7.0f}" for k, n in enumerate(names)))
    print("    sub-phases: " + "  ".join(f"{n} {acc[k, sl].mean():7.0f}" for k, n in enumerate(accn) if n != "-"))
