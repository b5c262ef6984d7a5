"""Python host binding of the HIP step engine (include/raftgpu.h) via ctypes.

This is the product path: it loads raftd_amd/libraftgpu.so and fails loudly if the library
is missing or no GPU is present. There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RAFTGPU_LIB") or os.path.join(PKG, "libraftgpu.so")  # override: experiments only
MAX_R = 8

RG_OK, RG_EINVAL, RG_ENOMEM, RG_EFULL, RG_EHIP, RG_EINVARIANT = 0, -1, -2, -3, -4, -5
RG_ERR_CRC, RG_ERR_MALFORMED, RG_ERR_POOL = 8, 32, 64  # rg_replica_view.err bits
TICK_NO_LOCALTICK = 1


class RgError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"raftgpu error {code}: {msg}")
        self.code = code


class Config(C.Structure):
    _fields_ = [
        ("groups", C.c_uint32), ("replicas", C.c_uint32), ("log_capacity", C.c_uint32),
        ("payload_bytes", C.c_uint32), ("max_entries_per_msg", C.c_uint32),
        ("max_msgs_per_pair", C.c_uint32), ("num_slabs", C.c_uint32),
        ("election_rtt", C.c_uint32), ("heartbeat_rtt", C.c_uint32), ("check_quorum", C.c_uint32),
        ("snapshot_entries", C.c_uint32), ("compaction_overhead", C.c_uint32),
        ("drop_ppm", C.c_uint32), ("device", C.c_int32), ("seed", C.c_uint64),
        ("ranks", C.c_uint32), ("rank", C.c_uint32), ("wire_all", C.c_uint32), ("column_base", C.c_uint32),
        ("crc32c", C.c_uint32), ("apply_feedback", C.c_uint32), ("initial_members", C.c_uint32),
        ("max_cmd_bytes", C.c_uint32), ("stream_pages", C.c_uint32), ("pool_pages", C.c_uint32),
        ("join_slots", C.c_uint32), ("wire_exact", C.c_uint32),
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
                ("crc", C.c_uint32), ("bank", C.c_uint32)]


class Traffic(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("replicas", "leaders", "msgs", "repl_entries", "appended",
                                          "leader_appended", "algorithmic_bytes", "bulk_bytes")]


class ApplyBatch(C.Structure):
    """rg_apply_batch: the committed entries as runs (rg_apply_run) + {len, crc} per entry + the Cmds."""
    _fields_ = [("runs", C.c_void_p), ("n_runs", C.c_uint64), ("cmds", C.c_void_p), ("n_entries", C.c_uint64),
                ("payload", C.c_void_p), ("payload_bytes", C.c_uint64)]


APPLY_RUN_DTYPE = np.dtype([("group", "<u8"), ("replica_id", "<u4"), ("rid", "<u4"), ("first", "<u8"),
                            ("entry", "<u8"), ("off", "<u8"), ("count", "<u4"), ("_pad", "<u4")])
APPLY_CMD_DTYPE = np.dtype([("len", "<u4"), ("crc", "<u4")])
# one row per entry, expanded on the host from the runs (what the drivers and tests consume)
APPLY_DTYPE = np.dtype([("index", "<u8"), ("group", "<u8"), ("replica_id", "<u4"), ("len", "<u4"),
                        ("crc", "<u4"), ("rid", "<u4"), ("off", "<u8")])


def expand_apply(runs, cmds):
    """APPLY_DTYPE rows (index, group, replica_id, len, crc, rid, off) from a batch's runs and per-entry
    {len, crc}: entry k of run r is index r.first + k, its Cmd at r.off + the 16-B-rounded lengths of
    the run's earlier entries (include/raftgpu.h, rg_apply_run)."""
    n = len(cmds)
    out = np.zeros(n, APPLY_DTYPE)
    if not n:
        return out
    cnt = runs["count"].astype(np.int64)
    rix = np.repeat(np.arange(len(runs)), cnt)
    k = np.arange(n, dtype=np.int64) - np.repeat(runs["entry"].astype(np.int64), cnt)
    out["index"] = runs["first"][rix] + k.astype(np.uint64)
    out["group"] = runs["group"][rix]
    out["replica_id"] = runs["replica_id"][rix]
    out["rid"] = runs["rid"][rix]
    out["len"] = cmds["len"]
    out["crc"] = cmds["crc"]
    rounded = (cmds["len"].astype(np.uint64) + 15) // 16 * 16
    excl = np.cumsum(rounded) - rounded  # exclusive prefix over the whole batch ...
    start = excl[runs["entry"].astype(np.int64)]  # ... minus the prefix at each run's first entry
    out["off"] = runs["off"][rix] + excl - start[rix]
    return out


def batch_arrays(b: "ApplyBatch", copy: bool = True):
    """(runs, cmds, payload) numpy arrays of an rg_apply_batch (views into engine-owned pinned memory
    unless copy)."""
    def arr(ptr, n, dt):
        if not n or not ptr:
            return np.zeros(0, dt)
        a = np.frombuffer((C.c_uint8 * (n * dt.itemsize)).from_address(ptr), dtype=dt)
        return a.copy() if copy else a
    return (arr(b.runs, b.n_runs, APPLY_RUN_DTYPE), arr(b.cmds, b.n_entries, APPLY_CMD_DTYPE),
            arr(b.payload, b.payload_bytes, np.dtype(np.uint8)))


PERSIST_STATE_DTYPE = np.dtype([("group", "<u8"), ("replica_id", "<u4"), ("rid", "<u4"), ("term", "<u8"),
                                ("vote", "<u8"), ("commit", "<u8"), ("last", "<u8"), ("marker", "<u8"),
                                ("marker_term", "<u8"), ("snap_index", "<u8"), ("snap_term", "<u8"),
                                ("first", "<u8"), ("entry_off", "<u8"), ("members", "<u4"), ("snap_members", "<u4"),
                                ("payload_off", "<u8"), ("term_off", "<u8"), ("n_terms", "<u4"), ("_pad", "<u4")])
PERSIST_CMD_DTYPE = np.dtype([("len", "<u4"), ("crc", "<u4")])  # rg_persist_entry
PERSIST_TERM_DTYPE = np.dtype([("term", "<u8"), ("count", "<u8")])  # rg_persist_term
PERSIST_CONFIG = 0x80000000  # RG_PERSIST_CONFIG
# one row per entry, expanded on the host from the ranges (what wal.py and the tests consume)
PERSIST_ENTRY_DTYPE = np.dtype([("index", "<u8"), ("term", "<u8"), ("type", "<u4"), ("len", "<u4"), ("crc", "<u4"),
                                ("rid", "<u4"), ("off", "<u8")])


class PersistBatch(C.Structure):
    """rg_persist_batch: per replica a state record, its entries as {len, crc}, their terms as runs,
    the Cmds packed."""
    _fields_ = [("states", C.c_void_p), ("n_states", C.c_uint64), ("entries", C.c_void_p), ("n_entries", C.c_uint64),
                ("terms", C.c_void_p), ("n_terms", C.c_uint64), ("payload", C.c_void_p), ("payload_bytes", C.c_uint64)]


def persist_arrays(b: "PersistBatch", copy: bool = True):
    """(states, entries, terms, payload) numpy arrays of an rg_persist_batch."""
    def arr(ptr, n, dt):
        if not n or not ptr:
            return np.zeros(0, dt)
        a = np.frombuffer((C.c_uint8 * (n * dt.itemsize)).from_address(ptr), dtype=dt)
        return a.copy() if copy else a
    return (arr(b.states, b.n_states, PERSIST_STATE_DTYPE), arr(b.entries, b.n_entries, PERSIST_CMD_DTYPE),
            arr(b.terms, b.n_terms, PERSIST_TERM_DTYPE), arr(b.payload, b.payload_bytes, np.dtype(np.uint8)))


def expand_persist(states, ents, terms):
    """PERSIST_ENTRY_DTYPE rows (index, term, type, len, crc, rid, off) from a persist batch's ranges:
    replica r's entry k is index r.first + k at entries[r.entry_off + k]; its term comes from the
    runs terms[r.term_off : r.term_off + r.n_terms]; its Cmd at r.payload_off + the 16-B-rounded
    lengths of the replica's earlier application entries (include/raftgpu.h, rg_persist_state)."""
    n = len(ents)
    out = np.zeros(n, PERSIST_ENTRY_DTYPE)
    if not n:
        return out
    fi, la = states["first"], states["last"]  # first > last (first may be ~0): no entries
    cnt = np.where(fi <= la, la - np.minimum(fi, la) + 1, 0).astype(np.int64)
    six = np.repeat(np.arange(len(states)), cnt)  # each entry's state record
    pos = np.arange(n, dtype=np.int64)
    k = pos - states["entry_off"].astype(np.int64)[six]
    out["index"] = states["first"][six] + k.astype(np.uint64)
    out["rid"] = states["rid"][six]
    out["term"] = np.repeat(terms["term"], terms["count"].astype(np.int64))
    cfg = (ents["len"] & PERSIST_CONFIG) != 0
    out["type"] = cfg.astype(np.uint32)
    out["len"] = ents["len"] & ~np.uint32(PERSIST_CONFIG)
    out["crc"] = ents["crc"]
    rounded = np.where(cfg, 0, (ents["len"].astype(np.uint64) + 15) // 16 * 16).astype(np.uint64)
    excl = np.cumsum(rounded) - rounded
    first_pos = states["entry_off"].astype(np.int64)[six]
    out["off"] = states["payload_off"][six] + excl - excl[first_pos]
    return out


ROW_CAP = 65536  # longest max_cmd_bytes shown as fixed-width rows; beyond it rows are as wide as the batch needs


def row_width(recs, max_cmd: int) -> int:
    """Row width of unpack_rows for a batch: max_cmd_bytes up to ROW_CAP (every batch the same shape),
    else the batch's longest Cmd rounded up to 16 B (a 16-MiB max_cmd_bytes would make every row 16 MiB)."""
    if max_cmd <= ROW_CAP or not len(recs):
        return max_cmd if max_cmd <= ROW_CAP else 0
    app = recs["type"] == 0 if "type" in recs.dtype.names else np.ones(len(recs), bool)
    m = int(recs["len"][app].max()) if app.any() else 0
    return (m + 15) // 16 * 16


def unpack_rows(recs, packed: np.ndarray, row: int) -> np.ndarray:
    """Packed Cmds (each at recs["off"], recs["len"] bytes) as one zero-padded row of `row` bytes per
    record: the Python view of rg_apply_committed / rg_persist_collect payloads."""
    out = np.zeros((len(recs), max(row, 1)), np.uint8)
    app = (recs["type"] == 0).tolist() if "type" in recs.dtype.names else [True] * len(recs)
    for k, (o, n) in enumerate(zip(recs["off"].tolist(), recs["len"].tolist())):
        if n and row and app[k]:  # a ConfigChange entry's len is its descriptor: no Cmd bytes
            out[k, :n] = packed[o:o + n]
    return out[:, :row]

SNAP_TAKEN, SNAP_RESTORED = 1, 2  # RG_SNAP_*
SNAPSHOT_EVENT_DTYPE = np.dtype([("group", "<u8"), ("replica_id", "<u4"), ("rid", "<u4"), ("kind", "<u4"),
                                 ("_pad", "<u4"), ("restored", "<u8"), ("index", "<u8"), ("term", "<u8")])


class Proposal(C.Structure):
    _fields_ = [("group", C.c_uint64), ("slot", C.c_uint32), ("count", C.c_uint32), ("first", C.c_uint64)]


def pack_proposals(batches):
    """[(global group, slot, [Cmd bytes, ...]), ...] → (rg_proposal array, u32 lens, packed u8 Cmd
    bytes): rg_propose's layout (Cmds back to back in lens order)."""
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


class ReadRequest(C.Structure):
    _fields_ = [("group", C.c_uint64), ("slot", C.c_uint32), ("_pad", C.c_uint32), ("ctx", C.c_uint64)]


READ_READY_DTYPE = np.dtype([("group", "<u8"), ("replica_id", "<u4"), ("rid", "<u4"), ("ctx", "<u8"), ("index", "<u8")])


_ALLGATHER = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_uint32)
_ALLTOALLV = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_void_p,
                         C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_void_p)


class Transport(C.Structure):
    """rg_transport (include/raftgpu.h): what rg_wire_exchange moves the regions with."""
    _fields_ = [("user", C.c_void_p), ("allgather_u64", _ALLGATHER), ("alltoallv", _ALLTOALLV)]


class Update(C.Structure):
    """rg_update (include/raftgpu.h): rg_get_update's sections, pointers into engine-owned pinned memory."""
    _fields_ = [("tick", C.c_uint64), ("persist", PersistBatch), ("committed", ApplyBatch), ("snapshots", C.c_void_p), ("n_snapshots", C.c_uint64),
                ("reads", C.c_void_p), ("n_reads", C.c_uint64), ("slot_mask", C.c_uint32), ("flags", C.c_uint32)]


UPDATE_PERSIST, UPDATE_COMMITTED, UPDATE_SNAPSHOTS, UPDATE_READS, UPDATE_ALL, UPDATE_FULL_STATE = 1, 2, 4, 8, 15, 16
UPDATE_COMMITTED_CMDS = 32  # ship the committed Cmds even with the persist section (no by-reference)


class PersistedCmds:
    """The host's copy of the Cmds an update stream persisted, kept until their replica applied them: what
    resolves rg_get_update's committed section when it comes by reference (RG_UPDATE_PERSIST together with
    RG_UPDATE_COMMITTED, include/raftgpu.h). dragonboat hands Update its entries from its own in-memory log
    the same way. Per replica {index: Cmd bytes}; a state record's window rewrites it (entries at or above
    its `first` are replaced, those above `last` dropped), an entry handed to the state machine is dropped
    with everything below it, and once the update is resolved the entries at or below each record's
    `marker` go too (compacted or restored past: a snapshot in the same step may compact entries that
    step also committed, so this comes after resolve)."""

    def __init__(self):
        self.log = {}

    def persist(self, states, entries, payload):
        for st in states:
            rid, first, last, marker = int(st["rid"]), int(st["first"]), int(st["last"]), int(st["marker"])
            d = self.log.setdefault(rid, {})
            for i in [i for i in d if i >= first or i > last]:
                del d[i]
        for e in entries:
            if e["type"] == 0:  # application entries (a ConfigChange carries no Cmd)
                o, n = int(e["off"]), int(e["len"])
                self.log.setdefault(int(e["rid"]), {})[int(e["index"])] = bytes(payload[o:o + n])

    def compact(self, states):
        for st in states:
            d = self.log.get(int(st["rid"]), {})
            marker = int(st["marker"])
            for i in [i for i in d if i <= marker]:
                del d[i]

    def resolve(self, runs, cmds):
        """The packed payload a by-reference committed section stands for: each Cmd at its run's off plus
        the 16-B-rounded lengths of the run's earlier entries (as rg_apply_committed would ship it)."""
        if not len(runs):
            return np.zeros(0, np.uint8)
        end = max(int(r["off"]) + sum((int(cmds[int(r["entry"]) + k]["len"]) + 15) // 16 * 16
                                      for k in range(int(r["count"]))) for r in runs)
        out = np.zeros(end, np.uint8)
        for r in runs:
            rid, first, at = int(r["rid"]), int(r["first"]), int(r["off"])
            d = self.log.get(rid, {})
            for k in range(int(r["count"])):
                n = int(cmds[int(r["entry"]) + k]["len"])
                cmd = d.get(first + k)
                if cmd is None or len(cmd) != n:
                    raise KeyError(f"committed entry {first + k} of replica {rid} was never persisted in this "
                                   f"update stream (RG_UPDATE_COMMITTED_CMDS ships it)")
                out[at:at + n] = np.frombuffer(cmd, np.uint8)
                at += (n + 15) // 16 * 16
            last = first + int(r["count"]) - 1
            for i in [i for i in d if i <= last]:  # handed to the state machine
                del d[i]
        return out
COMMIT_APPLIED = 1


class TickInput(C.Structure):
    _fields_ = [("prop_target", C.c_void_p), ("prop_count", C.c_void_p), ("campaign", C.c_void_p),
                ("isolate", C.c_void_p), ("flags", C.c_uint32), ("_pad", C.c_uint32)]


REPLICA_FIELDS = [f for f, _ in ReplicaView._fields_ if not f.startswith("_")]
CC_ADD, CC_REMOVE = 1, 2  # rg_config_change ops


def with_members(view: dict, R: int) -> dict:
    """A view for import: a dict without membership fields means every slot is a member."""
    if "members" not in view:
        view = dict(view, members=(1 << R) - 1)
    if "snap_members" not in view:
        view = dict(view, snap_members=view["members"])
    return view
MSG_FIELDS = [f for f, _ in MsgView._fields_]

# every symbol include/raftgpu.h declares
EXPORTS = ["rg_create", "rg_destroy", "rg_bootstrap", "rg_fill_slabs", "rg_tick", "rg_tick_device",
           "rg_set_stream", "rg_sync", "rg_tick_count", "rg_read_replicas", "rg_read_msgs",
           "rg_read_entries", "rg_import_replica", "rg_deliver", "rg_leader", "rg_sum_committed",
           "rg_device_bytes", "rg_last_error", "rg_last_tick_traffic", "rg_join",
           "rg_timing", "rg_kernel_ms", "rg_wire_plan", "rg_wire_pack", "rg_wire_pack_at", "rg_wire_recv", "rg_global_id",
           "rg_apply_committed", "rg_probe_copy", "rg_persist_collect", "rg_snapshot_events", "rg_propose",
           "rg_notify_applied", "rg_apply_async", "rg_apply_wait", "rg_read_index", "rg_read_index_results",
           "rg_config_change", "rg_wire_exchange", "rg_rccl_unique_id", "rg_rccl_open", "rg_rccl_close",
           "rg_pool_stats", "rg_get_update", "rg_commit_update", "rg_tick_device_n", "rg_digest",
           "rg_host_register", "rg_host_unregister", "rg_wire_plan_fixed", "rg_wire_dropped", "rg_compact",
           "rg_timing_epoch", "rg_kernel_events"]

_lib = None


def timing_epoch(device: int) -> None:
    """rg_timing_epoch: the process's reference event on `device`; launches timed afterwards by any
    engine there carry start / end times on that one timeline (Engine.kernel_events)."""
    rc = load_library().rg_timing_epoch(int(device))
    if rc != 0:
        raise RuntimeError(f"rg_timing_epoch: {load_library().rg_last_error().decode()}")


def load_library(path: str = LIB_PATH):
    """Load libraftgpu.so and declare signatures. Raises if it is missing (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process. PyTorch-ROCm wheels ship their own libamdhip64.so /
    # libhsa-runtime64.so (SONAMEs libamdhip64.so.7 / libhsa-runtime64.so.1) and libtorch_hip NEEDs
    # the unversioned name. If this library pulled /opt/rocm's runtime in first, a later torch
    # import would load the second copy and two HSA runtimes would share the process's KFD
    # context (observed: memory-aperture faults, "No HIP GPUs" at torch's lazy init). Importing
    # torch first lets the dynamic linker satisfy our libamdhip64.so.7 with torch's copy.
    try:
        import torch  # noqa: F401
    except ImportError:  # no torch (e.g. a cgo host): the system runtime is the only one
        pass
    if not os.path.exists(path):
        raise RuntimeError(f"HIP engine library not built: {path} (run `python -m raftd_amd.build`)")
    L = C.CDLL(path)
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
    sig = {
        "rg_create": ([C.POINTER(Config), C.POINTER(vp)], i32),
        "rg_destroy": ([vp], None),
        "rg_bootstrap": ([vp], i32),
        "rg_fill_slabs": ([vp], i32),
        "rg_tick": ([vp, C.POINTER(TickInput)], i32),
        "rg_tick_device": ([vp, C.POINTER(TickInput)], i32),
        "rg_tick_device_n": ([vp, C.POINTER(TickInput), u32, u32], i32),
        "rg_set_stream": ([vp, vp], i32),
        "rg_sync": ([vp], i32),
        "rg_join": ([vp], i32),
        "rg_timing": ([vp, i32], i32),
        "rg_kernel_ms": ([vp, C.POINTER(C.c_double), C.POINTER(C.c_uint64)], i32),
        "rg_timing_epoch": ([i32], i32),
        "rg_kernel_events": ([vp, i32, vp, vp, vp, u64, C.POINTER(C.c_uint64)], i32),
        "rg_tick_count": ([vp], u64),
        "rg_read_replicas": ([vp, u32, u32, C.POINTER(ReplicaView)], i32),
        "rg_read_msgs": ([vp, u32, u32, C.POINTER(MsgView), u32, C.POINTER(C.c_uint64)], i32),
        "rg_read_entries": ([vp, u32, u64, u32, C.POINTER(EntryView), vp], i32),
        "rg_import_replica": ([vp, u32, C.POINTER(ReplicaView), vp, vp, vp, vp], i32),
        "rg_propose": ([vp, C.POINTER(Proposal), C.c_size_t, vp, vp], i32),
        "rg_host_register": ([vp, vp, C.c_size_t], i32),
        "rg_host_unregister": ([vp, vp], i32),
        "rg_notify_applied": ([vp, vp, vp, C.c_size_t], i32),
        "rg_apply_async": ([vp, u32, i32], i32),
        "rg_read_index": ([vp, C.POINTER(ReadRequest), C.c_size_t], i32),
        "rg_config_change": ([vp, u64, u32, u32, u32], i32),
        "rg_compact": ([vp, u64, u64, C.POINTER(C.c_uint32)], i32),
        "rg_read_index_results": ([vp, u32, vp, u64, C.POINTER(C.c_uint64)], i32),
        "rg_apply_wait": ([vp, i32, vp], i32),
        "rg_deliver": ([vp, u32, C.POINTER(MsgView)], i32),
        "rg_leader": ([vp, u32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_int)], i32),
        "rg_sum_committed": ([vp, C.POINTER(C.c_uint64)], i32),
        "rg_device_bytes": ([vp], u64),
        "rg_last_tick_traffic": ([vp, C.POINTER(Traffic)], i32),
        "rg_last_error": ([], C.c_char_p),
        "rg_wire_plan": ([vp, C.POINTER(C.c_uint64)], i32),
        "rg_wire_plan_fixed": ([vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)], i32),
        "rg_wire_dropped": ([vp, C.POINTER(C.c_uint64)], i32),
        "rg_wire_pack": ([vp, vp, u64], i32),
        "rg_wire_pack_at": ([vp, vp, C.POINTER(C.c_uint64), u64], i32),
        "rg_wire_recv": ([vp, vp, C.POINTER(C.c_uint64)], i32),
        "rg_wire_exchange": ([vp, C.POINTER(Transport), C.POINTER(C.c_uint64)], i32),
        "rg_rccl_unique_id": ([C.c_char_p], i32),
        "rg_rccl_open": ([C.c_char_p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(Transport)], i32),
        "rg_rccl_close": ([C.POINTER(Transport)], i32),
        "rg_global_id": ([vp, u32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)], i32),
        "rg_apply_committed": ([vp, u32, vp], i32),
        "rg_pool_stats": ([vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_int)], i32),
        "rg_get_update": ([vp, u32, u32, C.POINTER(Update)], i32),
        "rg_digest": ([vp, C.POINTER(C.c_uint64)], i32),
        "rg_commit_update": ([vp, C.POINTER(Update), u32], i32),
        "rg_probe_copy": ([C.c_int32, u64, C.c_int32, C.POINTER(C.c_double)], i32),
        "rg_snapshot_events": ([vp, u32, vp, u64, C.POINTER(C.c_uint64)], i32),
        "rg_persist_collect": ([vp, i32, vp], i32),
    }
    for name, (args, res) in sig.items():
        if os.environ.get("RAFTGPU_LIB") and not hasattr(L, name):
            continue  # an experiment's library (ablations of an older build) may lack newer entry points
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def default_config(**kw) -> dict:
    """raftd's Raft parameters (raft/raft_manager.go:92-100) plus the engine's sizing."""
    c = dict(groups=4, replicas=3, log_capacity=2048, payload_bytes=256, max_entries_per_msg=64,
             max_msgs_per_pair=8, num_slabs=2, election_rtt=10, heartbeat_rtt=1, check_quorum=1,
             snapshot_entries=1000, compaction_overhead=5, drop_ppm=0, device=0, seed=0x5EED,
             ranks=1, rank=0, wire_all=0, column_base=0, crc32c=0, apply_feedback=0,
             initial_members=0, max_cmd_bytes=0, stream_pages=0, pool_pages=0, join_slots=0, wire_exact=0)
    c.update(kw)
    return c


class Engine:
    """One engine = the replicas one GPU hosts: with ranks = 1 every replica of `groups` Raft
    shards; with ranks = N the replicas placed on rank `rank` of N * groups shards.
    Local replica ids are column * R + slot; tick inputs are indexed by global group / replica."""

    def __init__(self, **cfg):
        self.cfg = default_config(**cfg)
        self.L = load_library()
        c = Config()
        for k, v in self.cfg.items():
            setattr(c, k, v)
        self.h = C.c_void_p()
        self._check(self.L.rg_create(C.byref(c), C.byref(self.h)))
        self.G, self.R = self.cfg["groups"], self.cfg["replicas"]
        self.nrep = self.G * self.R
        self.ranks = max(1, self.cfg["ranks"])
        self.row = self.cfg["max_cmd_bytes"] or self.cfg["payload_bytes"]  # longest Cmd: payload row stride
        self._slabs_filled = False

    def _check(self, rc):
        if rc < 0:
            raise RgError(rc, self.L.rg_last_error().decode())
        return rc

    def close(self):
        if getattr(self, "h", None):
            self.L.rg_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # lifecycle
    def bootstrap(self):
        self._check(self.L.rg_bootstrap(self.h))
        if not self._slabs_filled:
            self.fill_slabs()

    def fill_slabs(self):
        self._check(self.L.rg_fill_slabs(self.h))
        self._slabs_filled = True

    def tick(self, prop_target=None, prop_count=None, campaign=None, isolate=None, flags=0, threads=None):
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
        self._check(self.L.rg_tick(self.h, C.byref(ti)))

    def propose(self, batches):
        """Stage client commands for the next tick (rg_propose): batches = [(global group, slot,
        [Cmd bytes, ...]), ...]. Raises RgError (RG_EINVAL / RG_EFULL) and stages nothing on failure."""
        props, lens, blob = pack_proposals(batches)
        self._check(self.L.rg_propose(self.h, props, len(batches), blob.ctypes.data if blob.size else None,
                                      lens.ctypes.data if lens.size else None))

    def host_register(self, ptr: int, nbytes: int):
        """rg_host_register: page-lock a long-lived host buffer Cmds are staged in (DMA straight from it)."""
        self._check(self.L.rg_host_register(self.h, ptr, nbytes))

    def host_unregister(self, ptr: int):
        self._check(self.L.rg_host_unregister(self.h, ptr))

    def tick_device(self, prop_target_ptr=0, prop_count_ptr=0, campaign_ptr=0, isolate_ptr=0, flags=0):
        ti = TickInput(prop_target_ptr or None, prop_count_ptr or None, campaign_ptr or None,
                       isolate_ptr or None, flags, 0)
        self._check(self.L.rg_tick_device(self.h, C.byref(ti)))

    def tick_device_n(self, k, prop_target_ptr=0, prop_count_ptr=0, campaign_ptr=0, isolate_ptr=0, flags=0,
                      graph=True, resident=False):
        """rg_tick_device_n: k ticks with the same device-resident inputs; graph: one captured HIP graph
        of the k ticks per call (RG_TICKN_GRAPH); resident: one launch of the resident control kernel
        (RG_TICKN_RESIDENT, metadata-only engines)."""
        ti = TickInput(prop_target_ptr or None, prop_count_ptr or None, campaign_ptr or None,
                       isolate_ptr or None, flags, 0)
        mode = 2 if resident else (1 if graph else 0)
        self._check(self.L.rg_tick_device_n(self.h, C.byref(ti), k, mode))

    def set_stream(self, stream_handle: int):
        self._check(self.L.rg_set_stream(self.h, C.c_void_p(stream_handle)))

    def join(self):
        self._check(self.L.rg_join(self.h))

    def sync(self):
        self._check(self.L.rg_sync(self.h))

    def timing(self, enable: bool = True, bulk_only: bool = False, every: int = 1):
        """Per-launch HIP-event timing of control_kernel / bulk_kernel (measurement only);
        bulk_only: time bulk_kernel alone (two event records per tick instead of four); every: time
        only the ticks whose count is a multiple of it."""
        mode = (2 if bulk_only else 1) if enable else 0
        self._check(self.L.rg_timing(self.h, mode | (max(int(every), 1) << 8) if mode else 0))

    def kernel_ms(self) -> dict:
        """{'control': (total_ms, launches), 'bulk': (total_ms, launches)} since timing(True)."""
        ms = (C.c_double * 2)()
        n = (C.c_uint64 * 2)()
        self._check(self.L.rg_kernel_ms(self.h, ms, n))
        return {"control": (ms[0], n[0]), "bulk": (ms[1], n[1])}

    def kernel_events(self, kernel: str = "bulk"):
        """Timed launches since timing(True) as {tick, start, end} (ms after the process's
        rg_timing_epoch): launches of engines on different streams on one timeline."""
        import numpy as np
        k = 0 if kernel == "control" else 1
        n = C.c_uint64()
        self._check(self.L.rg_kernel_events(self.h, k, None, None, None, 0, C.byref(n)))
        ticks, a, b = np.zeros(n.value, np.uint64), np.zeros(n.value), np.zeros(n.value)
        self._check(self.L.rg_kernel_events(self.h, k, ticks.ctypes.data, a.ctypes.data, b.ctypes.data, n.value,
                                            C.byref(n)))
        return ticks, a, b

    @property
    def t(self) -> int:
        return self.L.rg_tick_count(self.h)

    @property
    def device_bytes(self) -> int:
        return self.L.rg_device_bytes(self.h)

    # views
    def replicas(self, first=0, n=None):
        n = self.nrep - first if n is None else n
        buf = (ReplicaView * n)()
        self._check(self.L.rg_read_replicas(self.h, first, n, buf))
        out = []
        for v in buf:
            d = {}
            for f in REPLICA_FIELDS:
                x = getattr(v, f)
                d[f] = list(x)[:self.R] if not isinstance(x, int) else x
            out.append(d)
        return out

    def replica(self, rid) -> dict:
        return self.replicas(rid, 1)[0]

    def replica_array(self, first=0, n=None):
        """rg_read_replicas as a numpy structured array (rg_replica_view fields), for bulk checks."""
        n = self.nrep - first if n is None else n
        buf = (ReplicaView * n)()
        self._check(self.L.rg_read_replicas(self.h, first, n, buf))
        return np.ctypeslib.as_array(buf).copy()

    def msgs(self, rid, dst) -> list:
        K, E = self.cfg["max_msgs_per_pair"], self.cfg["max_entries_per_msg"]
        buf = (MsgView * K)()
        terms = (C.c_uint64 * (K * E))()
        n = self._check(self.L.rg_read_msgs(self.h, rid, dst, buf, K, terms))
        out = []
        for k in range(n):
            m = buf[k]
            d = {("from" if f == "from_" else f): getattr(m, f) for f in MSG_FIELDS}
            d["terms"] = list(terms[k * E:k * E + m.nent]) if m.type == 12 else []
            out.append(d)
        return out

    def entries(self, rid, first, n, with_payload=False):
        if n <= 0:
            return []
        buf = (EntryView * n)()
        self._check(self.L.rg_read_entries(self.h, rid, first, n, buf, None))
        pay = None
        if with_payload and self.row:
            # rg_read_entries packs the application entries' Cmds back to back at their own lengths (a
            # ConfigChange entry's len is its descriptor, DESIGN.md §1.4: no Cmd bytes)
            tot = sum(ev.len for ev in buf if ev.type == 0)
            pay = (C.c_uint8 * max(tot, 1))()
            self._check(self.L.rg_read_entries(self.h, rid, first, n, buf, pay))
        out, at = [], 0
        for ev in buf:
            d = dict(term=ev.term, type=ev.type, len=ev.len, crc=ev.crc)
            if pay is not None:
                ln = ev.len if ev.type == 0 else 0
                d["payload"] = bytes(pay[at:at + ln])
                at += ln
            out.append(d)
        return out

    def entry(self, rid, index, with_payload=False):
        r = self.replica(rid)
        if not (r["marker"] < index <= r["last"]):
            return None
        return self.entries(rid, index, 1, with_payload)[0]

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
        self._check(self.L.rg_import_replica(self.h, rid, C.byref(v), t.ctypes.data if len(t) else None,
                                             None if ty is None else ty.ctypes.data,
                                             None if pl is None else pl.ctypes.data,
                                             None if ln is None or not ln.size else ln.ctypes.data))

    def deliver(self, rid_src, **fields):
        m = MsgView()
        for k, v in fields.items():
            setattr(m, "from_" if k == "from" else k, v)
        if "from" not in fields:
            m.from_ = rid_src % self.R + 1
        self._check(self.L.rg_deliver(self.h, rid_src, C.byref(m)))

    def read_index(self, reqs):
        """Stage ReadIndex requests [(global group, slot, ctx)] for the next tick (rg_read_index)."""
        arr = (ReadRequest * max(len(reqs), 1))()
        for i, (g, s, ctx) in enumerate(reqs):
            arr[i].group, arr[i].slot, arr[i].ctx = g, s, ctx
        self._check(self.L.rg_read_index(self.h, arr, len(reqs)))

    def read_index_results(self, slot_mask: int = 0xFF):
        """Reads made ready in the last tick (rg_read_index_results): READ_READY_DTYPE rows."""
        n = C.c_uint64()
        rc = self.L.rg_read_index_results(self.h, slot_mask, None, 0, C.byref(n))
        if rc < 0 and rc != RG_EFULL:
            self._check(rc)
        out = np.zeros(max(n.value, 1), READ_READY_DTYPE)
        self._check(self.L.rg_read_index_results(self.h, slot_mask, out.ctypes.data, n.value, C.byref(n)))
        return out[:n.value]

    def config_change(self, group, slot, op, target):
        """Stage a membership change for the next tick (rg_config_change): ConfigChange entry adding
        (CC_ADD) or removing (CC_REMOVE) slot `target` of global shard `group`, proposed at `slot`."""
        self._check(self.L.rg_config_change(self.h, group, slot, op, target))

    def read_ready_all(self) -> dict:
        """{local rid: [(ctx, index), ...]} for the reads made ready in the last tick, in order."""
        out = {}
        for r in self.read_index_results():
            out.setdefault(int(r["rid"]), []).append((int(r["ctx"]), int(r["index"])))
        return out

    def read_ready(self, rid):
        """[(ctx, index), ...] made ready for local replica rid in the last tick."""
        return self.read_ready_all().get(rid, [])

    def compact(self, group, index) -> int:
        """rg_compact: compact every local replica of global shard `group` to min(index, its snap_index);
        returns how many were compacted."""
        n = C.c_uint32()
        self._check(self.L.rg_compact(self.h, group, index, C.byref(n)))
        return n.value

    def notify_applied(self, rids, index):
        """rg_notify_applied (Peer.NotifyRaftLastApplied) for local replicas rids."""
        r = np.ascontiguousarray(np.atleast_1d(rids), dtype=np.uint32)
        i = np.ascontiguousarray(np.atleast_1d(index), dtype=np.uint64)
        assert r.shape == i.shape
        self._check(self.L.rg_notify_applied(self.h, r.ctypes.data, i.ctypes.data, r.size))

    def leader(self, group):
        lid, term, valid = C.c_uint64(), C.c_uint64(), C.c_int()
        self._check(self.L.rg_leader(self.h, group, C.byref(lid), C.byref(term), C.byref(valid)))
        return lid.value, term.value, bool(valid.value)

    def sum_committed(self) -> int:
        v = C.c_uint64()
        self._check(self.L.rg_sum_committed(self.h, C.byref(v)))
        return v.value

    # inter-rank exchange (include/raftgpu.h rg_wire_*)
    def wire_plan(self) -> list:
        out = (C.c_uint64 * self.ranks)()
        self._check(self.L.rg_wire_plan(self.h, out))
        return list(out)

    def wire_plan_fixed(self):
        """rg_wire_plan_fixed: (send capacities, receive capacities) per rank, agreed by both ends of
        every link without a size exchange; no host sync."""
        so, ro = (C.c_uint64 * self.ranks)(), (C.c_uint64 * self.ranks)()
        self._check(self.L.rg_wire_plan_fixed(self.h, so, ro))
        return list(so), list(ro)

    def wire_dropped(self) -> int:
        v = C.c_uint64()
        self._check(self.L.rg_wire_dropped(self.h, C.byref(v)))
        return v.value

    def wire_pack(self, send_ptr: int, send_cap: int):
        self._check(self.L.rg_wire_pack(self.h, C.c_void_p(send_ptr or None), send_cap))

    def wire_pack_at(self, base_ptr: int, region_off, base_cap: int):
        """rg_wire_pack_at: region r at base + region_off[r]."""
        ro = (C.c_uint64 * self.ranks)(*region_off)
        self._check(self.L.rg_wire_pack_at(self.h, C.c_void_p(base_ptr or None), ro, base_cap))

    def wire_recv(self, recv_ptr: int, recv_bytes):
        rb = (C.c_uint64 * self.ranks)(*recv_bytes)
        self._check(self.L.rg_wire_recv(self.h, C.c_void_p(recv_ptr or None), rb))

    def wire_exchange(self, transport: "Transport") -> int:
        """rg_wire_exchange: plan (fixed capacities unless the engine was made with wire_exact=1), pack,
        one transport all-to-all, unpack in one call (the C-ABI path a non-Python host uses; transport =
        rccl_transport(...) or PyTransport(...).t). Returns the bytes sent to other ranks."""
        sent = C.c_uint64()
        self._check(self.L.rg_wire_exchange(self.h, C.byref(transport), C.byref(sent)))
        return sent.value

    def apply_batch(self, slot_mask: int = 0xFF):
        """rg_apply_committed as the C-ABI returns it: (APPLY_RUN_DTYPE runs, APPLY_CMD_DTYPE per entry,
        packed Cmd bytes), numpy copies."""
        b = ApplyBatch()
        self._check(self.L.rg_apply_committed(self.h, slot_mask, C.byref(b)))
        return batch_arrays(b)

    def apply_committed_packed(self, slot_mask: int = 0xFF):
        """rg_apply_committed: (APPLY_DTYPE rows expanded from the runs, packed Cmd bytes, each at its
        row's off)."""
        runs, cmds, pay = self.apply_batch(slot_mask)
        return expand_apply(runs, cmds), pay

    def apply_committed(self, slot_mask: int = 0xFF):
        """Committed-entry copy-back of the last tick (rg_apply_committed): a structured array
        (APPLY_DTYPE: index, group, replica_id, len, crc, rid, off) and the Cmds, one zero-padded row per
        entry (row_width: max_cmd_bytes, or the batch's longest Cmd beyond ROW_CAP), as numpy arrays."""
        recs, packed = self.apply_committed_packed(slot_mask)
        return recs, unpack_rows(recs, packed, row_width(recs, self.row))

    def apply_async(self, slot_mask: int = 0xFF, buf: int = 0):
        """rg_apply_async: gather the last tick's applied entries and start their D2H copy into
        pinned buffer `buf` (0/1), overlapping the next ticks."""
        self._check(self.L.rg_apply_async(self.h, slot_mask, buf))

    def apply_wait(self, buf: int = 0, copy: bool = True):
        """rg_apply_wait: buffer `buf`'s batch. copy: (APPLY_DTYPE rows, Cmd rows) as numpy copies;
        copy=False: the raw (runs, cmds, packed payload) views into engine-owned pinned memory, valid
        until the next apply_async into `buf` (no host expansion: the measured path)."""
        b = ApplyBatch()
        self._check(self.L.rg_apply_wait(self.h, buf, C.byref(b)))
        if not copy:
            return batch_arrays(b, copy=False)
        runs, cmds, packed = batch_arrays(b)
        recs = expand_apply(runs, cmds)
        return recs, unpack_rows(recs, packed, row_width(recs, self.row))

    def persist_collect(self, full: bool = False):
        """Host WAL feed of the last tick (rg_persist_collect): (states, entries, payload) numpy
        arrays — PERSIST_STATE_DTYPE rows, PERSIST_ENTRY_DTYPE rows, one Cmd row per entry (row_width)."""
        b = PersistBatch()
        self._check(self.L.rg_persist_collect(self.h, 1 if full else 0, C.byref(b)))
        st, ents, terms, packed = persist_arrays(b)
        en = expand_persist(st, ents, terms)
        return st, en, unpack_rows(en, packed, row_width(en, self.row))

    def persist_batch(self, full: bool = False, copy: bool = True):
        """rg_persist_collect's ranges as (states, entries {len, crc}, term runs, payload) arrays."""
        b = PersistBatch()
        self._check(self.L.rg_persist_collect(self.h, 1 if full else 0, C.byref(b)))
        return persist_arrays(b, copy)

    def get_update(self, slot_mask: int = 0xFF, flags: int = UPDATE_ALL):
        """rg_get_update: the last tick's whole hand-off in one call. Returns (raw rg_update, dict of
        numpy copies: states, entries, entry_payload, committed, committed_payload, snapshots, reads).
        With the persist and committed sections together the committed Cmds come by reference (each
        crosses PCIe once) and are resolved from this engine's PersistedCmds (`committed_by_reference`):
        call it after every tick with the same slot mask, as a daemon's Update loop does."""
        u = Update()
        self._check(self.L.rg_get_update(self.h, slot_mask, flags, C.byref(u)))

        def arr(ptr, n, dt):
            if not n:
                return np.zeros(0, dt)
            return np.frombuffer((C.c_uint8 * (n * dt.itemsize)).from_address(ptr), dtype=dt).copy()

        st, ents, terms, epay = persist_arrays(u.persist)
        out = {"states": st, "entries": expand_persist(st, ents, terms), "entry_payload": epay,
               "persist_terms": terms, "committed": None, "committed_payload": None,
               "snapshots": arr(u.snapshots, u.n_snapshots, SNAPSHOT_EVENT_DTYPE),
               "reads": arr(u.reads, u.n_reads, READ_READY_DTYPE)}
        runs, cmds, out["committed_payload"] = batch_arrays(u.committed)
        by_ref = bool(u.committed.n_entries) and not u.committed.payload
        if flags & UPDATE_PERSIST:
            if not hasattr(self, "_persisted"):
                self._persisted = PersistedCmds()
            self._persisted.persist(st, out["entries"], epay)
        if by_ref:
            out["committed_payload"] = self._persisted.resolve(runs, cmds)
        if flags & UPDATE_PERSIST:
            self._persisted.compact(st)
        out["committed_by_reference"] = by_ref
        out["committed"] = expand_apply(runs, cmds)
        out["committed_runs"] = runs
        return u, out

    def commit_update(self, u, applied: bool = True):
        """rg_commit_update (Peer.Commit); applied: the slot mask's replicas report applied = processed."""
        self._check(self.L.rg_commit_update(self.h, C.byref(u), COMMIT_APPLIED if applied else 0))

    def digest(self):
        """rg_digest: (view digest, log digest) of this engine's replicas."""
        out = (C.c_uint64 * 2)()
        self._check(self.L.rg_digest(self.h, out))
        return out[0], out[1]

    def pool_stats(self) -> dict:
        """rg_pool_stats: {'total': pages, 'free': pages, 'failed': bool} of the payload page pool."""
        tot, free, failed = C.c_uint64(), C.c_uint64(), C.c_int()
        self._check(self.L.rg_pool_stats(self.h, C.byref(tot), C.byref(free), C.byref(failed)))
        return {"total": tot.value, "free": free.value, "failed": bool(failed.value)}

    def snapshot_events(self, slot_mask: int = 0xFF):
        """Snapshot events of the last tick (rg_snapshot_events): SNAPSHOT_EVENT_DTYPE rows, one
        per replica, in device order (slot by slot)."""
        n = C.c_uint64()
        rc = self.L.rg_snapshot_events(self.h, slot_mask, None, 0, C.byref(n))
        if rc < 0 and rc != RG_EFULL:
            self._check(rc)
        ev = np.zeros(max(n.value, 1), SNAPSHOT_EVENT_DTYPE)
        self._check(self.L.rg_snapshot_events(self.h, slot_mask, ev.ctypes.data, n.value, C.byref(n)))
        return ev[:n.value]

    def global_id(self, rid: int):
        """(global group, global replica id) of local replica rid."""
        g, gr = C.c_uint64(), C.c_uint64()
        self._check(self.L.rg_global_id(self.h, rid, C.byref(g), C.byref(gr)))
        return g.value, gr.value

    def last_tick_traffic(self) -> dict:
        t = Traffic()
        self._check(self.L.rg_last_tick_traffic(self.h, C.byref(t)))
        return {f: getattr(t, f) for f, _ in Traffic._fields_}


def rccl_unique_id() -> bytes:
    """rg_rccl_unique_id: 128 bytes rank 0 creates and hands to every rank out of band."""
    L = load_library()
    buf = C.create_string_buffer(128)
    if L.rg_rccl_unique_id(buf) != 0:
        raise RgError(-4, "rg_rccl_unique_id: librccl unavailable")
    return buf.raw


def rccl_transport(uid: bytes, nranks: int, rank: int, device: int = 0) -> Transport:
    """The library's built-in RCCL transport (rg_rccl_open); close with rccl_close(t)."""
    L = load_library()
    t = Transport()
    rc = L.rg_rccl_open(C.create_string_buffer(bytes(uid), 128), nranks, rank, device, C.byref(t))
    if rc != 0:
        raise RgError(rc, "rg_rccl_open failed")
    return t


def rccl_close(t: Transport):
    load_library().rg_rccl_close(C.byref(t))


class PyTransport:
    """An rg_transport whose callbacks are Python: allgather(list of n ints) -> list of ranks*n
    ints; alltoallv(send_ptr, soff, ssize, recv_ptr, roff, rsize, stream) moves device regions and
    must respect the ordering rule of include/raftgpu.h. Exceptions become a failed call."""

    def __init__(self, allgather, alltoallv):
        def ag(_user, mine, all_, n):
            try:
                vals = allgather([mine[i] for i in range(n)])
                for i, v in enumerate(vals):
                    all_[i] = v
                return 0
            except Exception as exc:  # noqa: BLE001 - reported through the C return code
                self.error = exc
                return -1

        def a2a(_user, send, soff, ssize, recv, roff, rsize, stream):
            try:
                k = self.nranks
                alltoallv(send or 0, [soff[i] for i in range(k)], [ssize[i] for i in range(k)], recv or 0,
                          [roff[i] for i in range(k)], [rsize[i] for i in range(k)], stream or 0)
                return 0
            except Exception as exc:  # noqa: BLE001
                self.error = exc
                return -1

        self.error = None
        self.nranks = 0
        self._cb = (_ALLGATHER(ag), _ALLTOALLV(a2a))  # keep the trampolines alive
        self.t = Transport(None, self._cb[0], self._cb[1])
