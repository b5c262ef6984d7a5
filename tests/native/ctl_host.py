"""ctypes wrapper of tests/native/ctl_host.cpp: the engine's control step on the CPU.

kind "ctl" in tests/engines.py. Entries expose term and type only (no payload: the bulk
kernel is not emulated), so comparisons against the oracle drop len/crc.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "build")


def build(asan: bool = False) -> str:
    os.makedirs(OUT, exist_ok=True)
    extra = os.environ.get("CTL_HOST_CFLAGS", "").split()  # ablations, e.g. -DRG_CTL_FASTREP
    tag = "".join(f.strip("-").replace("=", "") for f in extra)
    lib = os.path.join(OUT, ("libctl_host_asan" if asan else "libctl_host") + (f"_{tag}" if tag else "") + ".so")
    src = os.path.join(HERE, "ctl_host.cpp")
    deps = [src, os.path.join(ROOT, "raftd_amd", "csrc", "raftgpu_control.h"),
            os.path.join(ROOT, "raftd_amd", "csrc", "raftgpu_internal.h"), os.path.join(ROOT, "include", "raftgpu.h")]
    if os.path.exists(lib) and all(os.path.getmtime(d) <= os.path.getmtime(lib) for d in deps):
        return lib
    # build into a private file and rename it into place: parallel test workers (pytest -n) that find
    # the library stale at the same time never load one another's half-written output
    tmp = f"{lib}.{os.getpid()}.tmp"
    cmd = ["g++", "-O1" if asan else "-O2", "-g", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__",
           "-I/opt/rocm/include", *extra, src, "-o", tmp]
    if asan:
        cmd[1:1] = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"]
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib)
    return lib


class CtlHost:
    def __init__(self, asan: bool = False, fast: int = 0, **cfg):
        """fast: 0 the full step; 1 the fast step first (role-specialised, as control_fast_kernel), the
        full step for a lane it hands off; 2 the same with the small-engine latency build (LAT)."""
        from raftd_amd.engine import Config, MsgView, ReplicaView, default_config  # struct layouts only
        self._MsgView, self._ReplicaView = MsgView, ReplicaView
        self.cfg = default_config(**cfg)
        self.L = C.CDLL(build(asan))
        vp = C.c_void_p
        self.L.ch_create.restype = vp
        self.L.ch_create.argtypes = [C.POINTER(Config)]
        for n in ("ch_destroy", "ch_bootstrap"):
            getattr(self.L, n).argtypes = [vp]
        c = Config()
        for k, v in self.cfg.items():
            setattr(c, k, v)
        self.h = self.L.ch_create(C.byref(c))
        self.L.ch_set_fast.argtypes = [vp, C.c_int]
        self.L.ch_slow_lanes.argtypes = [vp]
        self.L.ch_slow_lanes.restype = C.c_uint64
        self.L.ch_violations.argtypes = [vp]
        self.L.ch_violations.restype = C.c_uint64
        self.L.ch_set_fast(C.c_void_p(self.h), int(fast))
        self.G, self.R = self.cfg["groups"], self.cfg["replicas"]
        self.nrep = self.G * self.R

    @property
    def slow_lanes(self) -> int:
        """Lanes the fast path handed to the full step so far (fast mode)."""
        return self.L.ch_slow_lanes(C.c_void_p(self.h))

    def close(self):
        if self.h:
            self.L.ch_destroy(C.c_void_p(self.h))
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def bootstrap(self):
        self.L.ch_bootstrap(C.c_void_p(self.h))

    def tick(self, prop_target=None, prop_count=None, campaign=None, isolate=None, flags=0, threads=None):
        from raftd_amd.engine import TickInput
        ti = TickInput()
        ti.flags = flags
        keep = []
        for name, arr, dt in (("prop_target", prop_target, np.uint8), ("prop_count", prop_count, np.uint32),
                              ("campaign", campaign, np.uint8), ("isolate", isolate, np.uint8)):
            if arr is None:
                setattr(ti, name, None)
            else:
                a = np.ascontiguousarray(arr, dtype=dt)
                keep.append(a)
                setattr(ti, name, a.ctypes.data)
        assert self.L.ch_tick(C.c_void_p(self.h), C.byref(ti)) == 0
        # the state is updated in place: a handed-off fast step must have left its rows untouched, and
        # the cached rows (S_LAST_TERM, S_NLPG, remote snapshot indices) must agree with what they cache
        assert self.L.ch_violations(C.c_void_p(self.h)) == 0, "ctl_host: in-place state invariant broken"

    def replica(self, rid) -> dict:
        from raftd_amd.engine import REPLICA_FIELDS
        v = self._ReplicaView()
        self.L.ch_read_replica(C.c_void_p(self.h), C.c_uint32(rid), C.byref(v))
        d = {}
        for f in REPLICA_FIELDS:
            x = getattr(v, f)
            d[f] = list(x)[:self.R] if not isinstance(x, int) else x
        return d

    def msgs(self, rid, dst) -> list:
        from raftd_amd.engine import MSG_FIELDS
        K, E = self.cfg["max_msgs_per_pair"], self.cfg["max_entries_per_msg"]
        buf = (self._MsgView * K)()
        terms = (C.c_uint64 * (K * E))()
        n = self.L.ch_read_msgs(C.c_void_p(self.h), C.c_uint32(rid), C.c_uint32(dst), buf, C.c_uint32(K), terms)
        out = []
        for k in range(n):
            m = buf[k]
            d = {("from" if f == "from_" else f): getattr(m, f) for f in MSG_FIELDS}
            d["terms"] = list(terms[k * E:k * E + m.nent]) if m.type == 12 else []
            out.append(d)
        return out

    def entry(self, rid, index, with_payload=False):
        r = self.replica(rid)
        if not (r["marker"] < index <= r["last"]):
            return None
        w = (C.c_uint64 * 1)()
        self.L.ch_read_words(C.c_void_p(self.h), C.c_uint32(rid), C.c_uint64(index), C.c_uint32(1), w)
        return dict(term=w[0] & ((1 << 36) - 1), type=(w[0] >> 61) & 1)  # raftgpu_internal.h TERM_MASK

    def import_replica(self, rid, view: dict, terms, types=None, payloads=None, lens=None):
        from raftd_amd.engine import REPLICA_FIELDS, with_members
        view = with_members(view, self.R)
        v = self._ReplicaView()
        for f in REPLICA_FIELDS:
            if f in view:
                x = view[f]
                if isinstance(x, (list, tuple)):
                    arr = getattr(v, f)
                    for i, y in enumerate(x):
                        arr[i] = y
                else:
                    setattr(v, f, x)
        t = np.ascontiguousarray(np.array(list(terms) + [0], dtype=np.uint64))
        ty = None if types is None else np.ascontiguousarray(np.array(types, dtype=np.uint32))
        ln = None if lens is None else np.ascontiguousarray(np.array(list(lens) + [0], dtype=np.uint32))
        self.L.ch_import(C.c_void_p(self.h), C.c_uint32(rid), C.byref(v), C.c_void_p(t.ctypes.data),
                         None if ty is None else C.c_void_p(ty.ctypes.data), C.c_int(1 if payloads is not None else 0),
                         None if ln is None else C.c_void_p(ln.ctypes.data))

    def read_index(self, reqs) -> int:
        """rg_read_index's staging on the CPU harness: [(group, slot, ctx), ...] (the caller validates)."""
        self.L.ch_read_index.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64]
        for g, s, ctx in reqs:
            self.L.ch_read_index(C.c_void_p(self.h), g * self.R + s, ctx)
        return 0

    def read_ready(self, rid):
        """[(ctx, index), ...] made ready for replica rid in the last tick."""
        c, i = (C.c_uint64 * 8)(), (C.c_uint64 * 8)()
        self.L.ch_read_ready.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint32]
        n = self.L.ch_read_ready(C.c_void_p(self.h), rid, c, i, 8)
        return [(c[k], i[k]) for k in range(n)]

    def feed(self, rid) -> dict:
        """Replica rid's hand-off word of the last step, decoded as the device's rg_get_update kernels
        decode it (raftgpu_internal.h feed_*)."""
        out = (C.c_uint64 * 5)()
        self.L.ch_feed.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
        assert self.L.ch_feed(C.c_void_p(self.h), rid, out) == 0
        return dict(apply_lo=out[0], restored=out[1], took=bool(out[2]), persist=bool(out[3]), persist_lo=out[4])

    def config_change(self, group, slot, op, target) -> int:
        """rg_config_change's staging on the CPU harness (the caller validates)."""
        fn = self.L.ch_config_change
        fn.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
        return fn(C.c_void_p(self.h), group, slot, op, target)

    def deliver(self, rid_src, **fields):
        m = self._MsgView()
        for k, v in fields.items():
            setattr(m, "from_" if k == "from" else k, v)
        assert self.L.ch_deliver(C.c_void_p(self.h), C.c_uint32(rid_src), C.byref(m)) == 0
