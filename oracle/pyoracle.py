"""ctypes wrapper over oracle/build/liboracle.so (the C restatement).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg. Parity against dragonboat is unpinned (see oracle/oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

MAX_R = 8

# message / role / state constants (oracle.h)
LOCAL_TICK, ELECTION, LEADER_HEARTBEAT, NOOP, PROPOSE = 0, 1, 2, 4, 7
CHECK_QUORUM, REPLICATE, REPLICATE_RESP, REQUEST_VOTE, REQUEST_VOTE_RESP = 10, 12, 13, 14, 15
INSTALL_SNAPSHOT, HEARTBEAT, HEARTBEAT_RESP = 16, 17, 18
FOLLOWER, CANDIDATE, LEADER = 0, 1, 2
RETRY, WAIT, REPLICATE_ST, SNAPSHOT = 0, 1, 2, 3
TICK_NO_LOCALTICK = 1


class Config(C.Structure):
    _fields_ = [
        ("groups", C.c_uint32), ("replicas", C.c_uint32), ("log_capacity", C.c_uint32),
        ("payload_bytes", C.c_uint32), ("max_entries_per_msg", C.c_uint32),
        ("max_msgs_per_pair", C.c_uint32), ("num_slabs", C.c_uint32),
        ("election_rtt", C.c_uint32), ("heartbeat_rtt", C.c_uint32), ("check_quorum", C.c_uint32),
        ("snapshot_entries", C.c_uint32), ("compaction_overhead", C.c_uint32),
        ("drop_ppm", C.c_uint32), ("group_base", C.c_uint32), ("seed", C.c_uint64),
        ("crc32c", C.c_uint32), ("apply_feedback", C.c_uint32), ("initial_members", C.c_uint32),
        ("max_cmd_bytes", C.c_uint32), ("stream_pages", C.c_uint32), ("join_slots", C.c_uint32),
        ("_pad", C.c_uint32),
    ]


class ReplicaView(C.Structure):
    _fields_ = [
        ("term", C.c_uint64), ("vote", C.c_uint64), ("leader", C.c_uint64),
        ("committed", C.c_uint64), ("applied", C.c_uint64), ("last", C.c_uint64),
        ("marker", C.c_uint64), ("marker_term", C.c_uint64), ("snap_index", C.c_uint64),
        ("snap_term", C.c_uint64), ("cap_base", C.c_uint64), ("processed", C.c_uint64),
        ("role", C.c_uint32), ("election_tick", C.c_uint32), ("heartbeat_tick", C.c_uint32),
        ("rand_timeout", C.c_uint32), ("rng_ctr", C.c_uint32), ("granted", C.c_uint32),
        ("responded", C.c_uint32), ("active", C.c_uint32), ("err", C.c_uint32), ("drops", C.c_uint32),
        ("members", C.c_uint32), ("snap_members", C.c_uint32), ("cc_pending", C.c_uint32), ("_mpad", C.c_uint32),
        ("match", C.c_uint64 * MAX_R), ("next", C.c_uint64 * MAX_R), ("rsnap", C.c_uint64 * MAX_R),
        ("rstate", C.c_uint8 * MAX_R),
    ]


class MsgView(C.Structure):
    _fields_ = [
        ("type", C.c_uint8), ("from_", C.c_uint8), ("to", C.c_uint8), ("reject", C.c_uint8),
        ("nent", C.c_uint32), ("term", C.c_uint64), ("log_term", C.c_uint64),
        ("log_index", C.c_uint64), ("commit", C.c_uint64), ("hint", C.c_uint64),
        ("hint_high", C.c_uint64), ("src_a", C.c_uint32), ("src_b", C.c_uint32),
    ]


class EntryView(C.Structure):
    _fields_ = [("term", C.c_uint64), ("type", C.c_uint32), ("len", C.c_uint32),
                ("crc", C.c_uint32), ("_pad", C.c_uint32)]


class Proposal(C.Structure):
    _fields_ = [("group", C.c_uint64), ("slot", C.c_uint32), ("count", C.c_uint32), ("first", C.c_uint64)]


class ReadRequest(C.Structure):
    _fields_ = [("group", C.c_uint64), ("slot", C.c_uint32), ("_pad", C.c_uint32), ("ctx", C.c_uint64)]


class TickInput(C.Structure):
    _fields_ = [("prop_target", C.c_void_p), ("prop_count", C.c_void_p), ("campaign", C.c_void_p),
                ("isolate", C.c_void_p), ("flags", C.c_uint32)]


REPLICA_FIELDS = [f for f, _ in ReplicaView._fields_ if not f.startswith("_")]
CONFIG_KEYS = {f for f, _ in Config._fields_}
CC_ADD, CC_REMOVE = 1, 2  # OR_CC_ADD / OR_CC_REMOVE


def with_members(view: dict, R: int) -> dict:
    """A view for import: a dict without membership fields means every slot is a member."""
    if "members" not in view:
        view = dict(view, members=(1 << R) - 1)
    if "snap_members" not in view:
        view = dict(view, snap_members=view["members"])
    return view
MSG_FIELDS = [f for f, _ in MsgView._fields_]


def build(quiet: bool = True) -> str:
    subprocess.run(["make", "-C", HERE], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
        L.or_create.argtypes = [C.POINTER(Config), C.POINTER(vp)]
        L.or_destroy.argtypes = [vp]
        L.or_bootstrap.argtypes = [vp]
        L.or_tick.argtypes = [vp, C.POINTER(TickInput), C.c_int]
        L.or_tick_count.argtypes = [vp]
        L.or_tick_count.restype = u64
        L.or_get_replica.argtypes = [vp, u32, C.POINTER(ReplicaView)]
        L.or_digest.argtypes = [vp, C.POINTER(C.c_uint64)]
        L.or_get_replicas.argtypes = [vp, u32, u32, C.POINTER(ReplicaView)]
        L.or_get_msgs.argtypes = [vp, u32, u32, C.POINTER(MsgView), u32]
        L.or_get_msg_terms.argtypes = [vp, u32, u32, u32, C.POINTER(C.c_uint64), u32]
        L.or_get_entry.argtypes = [vp, u32, u64, C.POINTER(EntryView), C.c_void_p]
        L.or_get_applied.argtypes = [vp, u32, C.c_void_p, C.c_void_p, C.c_void_p, u32]
        L.or_get_snapshot_event.argtypes = [vp, u32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                            C.POINTER(C.c_uint64)]
        L.or_debug_apply_lo.argtypes = [vp, u32, C.POINTER(C.c_uint64)]
        L.or_import_replica.argtypes = [vp, u32, C.POINTER(ReplicaView), C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p]
        L.or_propose.argtypes = [vp, C.POINTER(Proposal), C.c_size_t, C.c_void_p, C.c_void_p]
        L.or_notify_applied.argtypes = [vp, u32, u64]
        L.or_config_change.argtypes = [vp, u64, u32, u32, u32]
        L.or_compact.argtypes = [vp, u64, u64]
        L.or_read_index.argtypes = [vp, C.POINTER(ReadRequest), C.c_size_t]
        L.or_get_read_ready.argtypes = [vp, u32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), u32]
        L.or_tick.restype = C.c_int
        L.or_deliver.argtypes = [vp, u32, C.POINTER(MsgView)]
        L.or_payload.argtypes = [vp, u32, u32, u32, C.c_void_p]
        L.or_crc32.argtypes = [C.c_void_p, C.c_size_t]
        L.or_crc32.restype = u32
        L.or_crc32c.argtypes = [C.c_void_p, C.c_size_t]
        L.or_crc32c.restype = u32
        L.or_mix64.argtypes = [u64]
        L.or_mix64.restype = u64
        _lib = L
    return _lib


def default_config(**kw) -> dict:
    """raftd's Raft parameters (raft/raft_manager.go:92-100) plus the engine's sizing."""
    c = dict(groups=4, replicas=3, log_capacity=2048, payload_bytes=256, max_entries_per_msg=64,
             max_msgs_per_pair=8, num_slabs=2, election_rtt=10, heartbeat_rtt=1, check_quorum=1,
             snapshot_entries=1000, compaction_overhead=5, drop_ppm=0, seed=0x5EED, group_base=0, crc32c=0,
             apply_feedback=0, initial_members=0, max_cmd_bytes=0, stream_pages=0, join_slots=0)
    c.update(kw)
    return c


def max_cmd(cfg: dict) -> int:
    """The longest Cmd of a configuration: max_cmd_bytes, or payload_bytes."""
    return cfg.get("max_cmd_bytes", 0) or cfg["payload_bytes"]


def make_config(d: dict) -> Config:
    c = Config()
    for k, v in d.items():
        setattr(c, k, v)
    return c


def view_to_dict(v) -> dict:
    out = {}
    for f in REPLICA_FIELDS:
        x = getattr(v, f)
        out[f] = list(x) if not isinstance(x, int) else x
    return out


def msg_to_dict(m) -> dict:
    return {("from" if f == "from_" else f): getattr(m, f) for f in MSG_FIELDS}


class TickInputs:
    """Keeps numpy buffers alive for one tick call."""

    def __init__(self, groups, replicas, prop_target=None, prop_count=None, campaign=None,
                 isolate=None, flags=0):
        self.bufs = []
        self.ti = TickInput()
        self.ti.flags = flags
        for name, arr, dt in (("prop_target", prop_target, np.uint8), ("prop_count", prop_count, np.uint32),
                              ("campaign", campaign, np.uint8), ("isolate", isolate, np.uint8)):
            if arr is None:
                setattr(self.ti, name, None)
            else:
                a = np.ascontiguousarray(arr, dtype=dt)
                self.bufs.append(a)
                setattr(self.ti, name, a.ctypes.data)


class Oracle:
    def __init__(self, **cfg):
        self.cfg = default_config(**cfg)
        self.L = lib()
        self.h = C.c_void_p()
        rc = self.L.or_create(C.byref(make_config({k: v for k, v in self.cfg.items() if k in CONFIG_KEYS})),
                              C.byref(self.h))
        if rc != 0:
            raise ValueError(f"or_create rejected config {self.cfg}")
        self.G, self.R = self.cfg["groups"], self.cfg["replicas"]
        self.nrep = self.G * self.R

    def close(self):
        if self.h:
            self.L.or_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def bootstrap(self):
        self.L.or_bootstrap(self.h)

    def tick(self, prop_target=None, prop_count=None, campaign=None, isolate=None, flags=0, threads=1):
        ti = TickInputs(self.G, self.R, prop_target, prop_count, campaign, isolate, flags)
        if self.L.or_tick(self.h, C.byref(ti.ti), threads) != 0:
            raise ValueError("or_tick: tick-input proposals while caller proposals are staged")

    def propose(self, batches):
        """Stage caller proposals for the next tick (or_propose): batches = [(global group, slot,
        [Cmd bytes, ...]), ...]. Returns the oracle's code (0, -1 invalid, -3 batch full)."""
        props, lens, blob = pack_proposals(batches)
        return self.L.or_propose(self.h, props, len(batches), blob.ctypes.data if blob.size else None,
                                 lens.ctypes.data if lens.size else None)

    @property
    def t(self) -> int:
        return self.L.or_tick_count(self.h)

    def replica(self, rid) -> dict:
        v = ReplicaView()
        assert self.L.or_get_replica(self.h, rid, C.byref(v)) == 0
        d = view_to_dict(v)
        R = self.R
        for f in ("match", "next", "rsnap", "rstate"):
            d[f] = d[f][:R]
        return d

    def replica_array(self, first=0, n=None):
        """Views of replicas first .. first+n-1 as a numpy structured array (bulk comparisons)."""
        n = self.nrep - first if n is None else n
        buf = (ReplicaView * n)()
        assert self.L.or_get_replicas(self.h, first, n, buf) == 0
        return np.ctypeslib.as_array(buf).copy()

    def msgs(self, rid, dst) -> list:
        buf = (MsgView * 16)()
        n = self.L.or_get_msgs(self.h, rid, dst, buf, 16)
        out = []
        for k in range(n):
            d = msg_to_dict(buf[k])
            terms = (C.c_uint64 * 64)()
            nt = self.L.or_get_msg_terms(self.h, rid, dst, k, terms, 64)
            d["terms"] = list(terms[:max(nt, 0)])
            out.append(d)
        return out

    def entry(self, rid, index, with_payload=False):
        ev = EntryView()
        rc = self.L.or_get_entry(self.h, rid, index, C.byref(ev), None)
        if rc != 0:
            return None
        d = dict(term=ev.term, type=ev.type, len=ev.len, crc=ev.crc)
        if with_payload and self.cfg["payload_bytes"]:
            if ev.type == 0 and ev.len:  # ConfigChange: len = descriptor, no Cmd
                pay = (C.c_uint8 * ev.len)()
                self.L.or_get_entry(self.h, rid, index, C.byref(ev), pay)
                d["payload"] = bytes(pay)
            else:
                d["payload"] = b""
        return d

    def applied_entries(self, rid):
        """Non-empty application entries rid handed to the state machine in the last step:
        [(index, len, crc, payload)] in index order (oracle side of rg_apply_committed)."""
        n = self.L.or_get_applied(self.h, rid, None, None, None, 0)
        if n <= 0:
            return []
        idx = (C.c_uint64 * n)()
        ev = (EntryView * n)()
        self.L.or_get_applied(self.h, rid, idx, ev, None, n)
        tot = sum(ev[k].len for k in range(n))
        pay = (C.c_uint8 * max(1, tot))()  # the Cmds, packed
        self.L.or_get_applied(self.h, rid, idx, ev, pay, n)
        out, at = [], 0
        for k in range(n):
            out.append((idx[k], ev[k].len, ev[k].crc, bytes(pay[at:at + ev[k].len])))
            at += ev[k].len
        return out

    def apply_lo(self, rid):
        """The first index rid's last step handed to the state machine (its apply window's start)."""
        v = C.c_uint64()
        assert self.L.or_debug_apply_lo(self.h, rid, C.byref(v)) == 0
        return v.value

    def snapshot_event(self, rid):
        """(kind, restored, index, term) of rid's last step (oracle side of rg_snapshot_events)."""
        r, i, t = C.c_uint64(), C.c_uint64(), C.c_uint64()
        k = self.L.or_get_snapshot_event(self.h, rid, C.byref(r), C.byref(i), C.byref(t))
        return k, r.value, i.value, t.value

    def log_terms(self, rid):
        r = self.replica(rid)
        return [self.entry(rid, i)["term"] for i in range(r["marker"] + 1, r["last"] + 1)]

    def import_replica(self, rid, view: dict, terms, types=None, payloads=None, lens=None):
        view = with_members(view, self.R)
        v = ReplicaView()
        for f in REPLICA_FIELDS:
            if f in view:
                x = view[f]
                if isinstance(x, (list, tuple)):
                    arr = getattr(v, f)
                    for i, y in enumerate(x):
                        arr[i] = y
                else:
                    setattr(v, f, x)
        t = np.ascontiguousarray(np.array(terms, dtype=np.uint64))
        ty = None if types is None else np.ascontiguousarray(np.array(types, dtype=np.uint32))
        pl = None if payloads is None else np.ascontiguousarray(np.frombuffer(payloads, dtype=np.uint8))
        ln = None if lens is None else np.ascontiguousarray(np.array(lens, dtype=np.uint32))
        rc = self.L.or_import_replica(self.h, rid, C.byref(v), t.ctypes.data if len(t) else None,
                                      None if ty is None else ty.ctypes.data,
                                      None if pl is None else pl.ctypes.data,
                                      None if ln is None or not ln.size else ln.ctypes.data)
        if rc != 0:
            raise ValueError("or_import_replica failed")

    def read_index(self, reqs) -> int:
        """Stage ReadIndex requests [(global group, slot, ctx)] for the next tick (or_read_index)."""
        arr = (ReadRequest * max(len(reqs), 1))()
        for i, (g, s, ctx) in enumerate(reqs):
            arr[i].group, arr[i].slot, arr[i].ctx = g, s, ctx
        return self.L.or_read_index(self.h, arr, len(reqs))

    def digest(self):
        """or_digest: (view digest, log digest) of every replica."""
        out = (C.c_uint64 * 2)()
        self.L.or_digest(self.h, out)
        return out[0], out[1]

    def read_ready(self, rid):
        """[(ctx, index), ...] of the reads replica rid made ready in the last tick, in order."""
        c, i = (C.c_uint64 * 8)(), (C.c_uint64 * 8)()
        n = self.L.or_get_read_ready(self.h, rid, c, i, 8)
        return [(c[k], i[k]) for k in range(n)]

    def compact(self, group, index) -> int:
        """or_compact (rg_compact): compact every replica of global shard `group` to min(index, its
        snap_index); returns the number compacted, -1 for a shard outside the engine."""
        return self.L.or_compact(self.h, group, index)

    def config_change(self, group, slot, op, target) -> int:
        """Stage a membership change for the next tick (or_config_change): 0, -1 invalid, -3 one
        already staged for the shard."""
        return self.L.or_config_change(self.h, group, slot, op, target)

    def notify_applied(self, rid, index) -> int:
        """or_notify_applied (Peer.NotifyRaftLastApplied): 0, or -1 if index > processed."""
        return self.L.or_notify_applied(self.h, rid, index)

    def deliver(self, rid_src, **fields):
        m = MsgView()
        for k, v in fields.items():
            setattr(m, "from_" if k == "from" else k, v)
        if "from" not in fields:
            m.from_ = rid_src % self.R + 1
        rc = self.L.or_deliver(self.h, rid_src, C.byref(m))
        if rc != 0:
            raise ValueError("or_deliver failed")

    def payload(self, slab, group, entry) -> bytes:
        buf = (C.c_uint8 * max(self.cfg["payload_bytes"], 1))()
        self.L.or_payload(self.h, slab, group, entry, buf)
        return bytes(buf[:self.cfg["payload_bytes"]])


def pack_proposals(batches):
    """[(group, slot, [cmd bytes])] → (Proposal array, u32 lens, packed u8 Cmd bytes): the layout
    or_propose and rg_propose take (Cmds back to back in lens order)."""
    props = (Proposal * max(len(batches), 1))()
    lens, chunks, first = [], [], 0
    for i, (g, s, cmds) in enumerate(batches):
        props[i].group, props[i].slot, props[i].count, props[i].first = g, s, len(cmds), first
        for c in cmds:
            lens.append(len(c))
            chunks.append(bytes(c))
        first += len(cmds)
    blob = np.frombuffer(b"".join(chunks), dtype=np.uint8).copy() if chunks else np.zeros(0, np.uint8)
    return props, np.array(lens, dtype=np.uint32), blob


def crc32(b: bytes) -> int:
    buf = C.create_string_buffer(b, len(b))
    return lib().or_crc32(buf, len(b))


def crc32c(b: bytes) -> int:
    buf = C.create_string_buffer(b, len(b))
    return lib().or_crc32c(buf, len(b))


def mix64(z: int) -> int:
    return lib().or_mix64(z & 0xFFFFFFFFFFFFFFFF)
