"""Host write-ahead log for the step engine: durability stays on the host.

dragonboat makes each step's ``Update.EntriesToSave`` and ``pb.State{Term, Vote, Commit}`` (plus a
snapshot's index and term) durable in its LogDB with fsync before the step's messages leave
(``SaveRaftState``; raftd keeps it under ``RAFT_DIR/node<ID>``, /root/reference/raft/raft_manager.go
:101-106), and a restarted NodeHost rebuilds every replica from it. Here, after each tick,
``rg_persist_collect`` hands over exactly that for every replica whose log or hard state changed
(one ``hipMemcpyAsync`` per array), ``WAL.append`` writes it as one framed, CRC-checked record and
fsyncs, and the engine may then run the next tick (which delivers the last tick's messages).

Record: ``b"RGWL"``, u32 version, u64 tick, u64 #states, u64 #entries, u32 row bytes (the record's
Cmd row width), u32 crc32(body), u64 len(body); body = the state rows, the entry rows, the Cmds, one
zero-padded row per entry (``PERSIST_STATE_DTYPE`` / ``PERSIST_ENTRY_DTYPE`` little-endian). A torn tail record
(crash mid-write: short, or failing its CRC) is ignored on replay; a complete record of another
format version is an error, never silently dropped.

Replay applies records in order per replica: keep the entries below ``first``, replace
``first..last`` with the record's entries, drop those above ``last`` and at or below ``marker``.
Restart (``restart_view``) is dragonboat's: the persisted State and log, the snapshot's index /
term as the compaction marker, the state machine caught up to Commit (raftd's ``Open`` returns
the application's last applied index), then ``becomeFollower(term, NoLeader)`` — volatile fields
reset, a fresh randomized election timeout (DESIGN.md §1.3 with the counter at 1). Messages in
flight at the crash are lost, as they are when a node dies.
"""
from __future__ import annotations

import os
import struct
import zlib

import numpy as np

from .engine import PERSIST_ENTRY_DTYPE, PERSIST_STATE_DTYPE

MAGIC = b"RGWL"
VERSION = 3  # 2: state records carry the membership (members, snap_members); 3: entry rows carry `off`
HDR = struct.Struct("<4sIQQQIIQ")


class WAL:
    def __init__(self, path: str, sync: bool = True):
        self.path, self.sync = path, sync
        self.f = open(path, "ab")

    def append(self, tick: int, states, entries, payload, payload_bytes: int | None = None):
        """payload: one zero-padded Cmd row per entry (Engine.persist_collect); its row width is
        recorded in the header (payload_bytes, if given, must match it)."""
        payload = np.ascontiguousarray(payload)
        row = int(payload.shape[1]) if payload.ndim == 2 else 0
        if payload_bytes is not None and len(entries) and row not in (payload_bytes, 0):
            raise ValueError(f"WAL.append: payload rows of {row} B, not {payload_bytes} B")
        body = states.tobytes() + entries.tobytes() + payload.tobytes()
        self.f.write(HDR.pack(MAGIC, VERSION, tick, len(states), len(entries), row,
                              zlib.crc32(body), len(body)))
        self.f.write(body)
        self.f.flush()
        if self.sync:
            os.fsync(self.f.fileno())
        return HDR.size + len(body)

    def close(self):
        self.f.close()


def records(path: str):
    """Yield (tick, states, entries, payload) for every intact record."""
    with open(path, "rb") as f:
        data = f.read()
    pos = 0
    while pos + HDR.size <= len(data):
        magic, ver, tick, ns, ne, P, crc, blen = HDR.unpack_from(data, pos)
        if magic != MAGIC or pos + HDR.size + blen > len(data):
            break  # torn tail
        if ver != VERSION:
            raise ValueError(f"WAL {path}: a record of format version {ver} at byte {pos}; this build reads "
                             f"version {VERSION} (replay it with the build that wrote it)")
        body = data[pos + HDR.size:pos + HDR.size + blen]
        if zlib.crc32(body) != crc:
            break
        sb, eb = ns * PERSIST_STATE_DTYPE.itemsize, ne * PERSIST_ENTRY_DTYPE.itemsize
        states = np.frombuffer(body[:sb], PERSIST_STATE_DTYPE)
        entries = np.frombuffer(body[sb:sb + eb], PERSIST_ENTRY_DTYPE)
        payload = np.frombuffer(body[sb + eb:], np.uint8).reshape(ne, P) if P else np.zeros((ne, 0), np.uint8)
        yield tick, states, entries, payload
        pos += HDR.size + blen


class ReplicaLog:
    """One replica's durable state: the last State record and its log (index → entry)."""

    __slots__ = ("state", "log")

    def __init__(self):
        self.state = None
        self.log = {}

    def apply(self, st, ents, pay):
        first, last, marker = int(st["first"]), int(st["last"]), int(st["marker"])
        for i in [i for i in self.log if i >= first or i > last or i <= marker]:
            del self.log[i]
        for k, e in enumerate(ents):
            i = int(e["index"])
            if marker < i <= last:
                self.log[i] = (int(e["term"]), int(e["type"]), int(e["len"]), int(e["crc"]),
                               bytes(pay[k, :int(e["len"])]))
        self.state = {n: int(st[n]) for n in PERSIST_STATE_DTYPE.names}


def replay(path: str, replicas: int) -> dict:
    """{global replica id: ReplicaLog} from every intact record of a WAL file."""
    out = {}
    for _, states, entries, payload in records(path):
        for st in states:
            gr = int(st["group"]) * replicas + int(st["replica_id"]) - 1
            lo, n = int(st["entry_off"]), max(0, int(st["last"]) - int(st["first"]) + 1)
            out.setdefault(gr, ReplicaLog()).apply(st, entries[lo:lo + n], payload[lo:lo + n])
    return out


def mix64(z: int) -> int:
    m = (1 << 64) - 1
    z ^= z >> 30
    z = (z * 0xBF58476D1CE4E5B9) & m
    z ^= z >> 27
    z = (z * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def restart_view(rl: ReplicaLog, group: int, slot: int, cfg: dict, app_applied=None) -> dict:
    """The replica view a restarted node starts from (becomeFollower(term, NoLeader)).

    applied = processed = the index the state machine reports as applied (raftd's Open returns the
    app's /LastLogIndex, raft/state_machine.go:101-124), at least the snapshot index (the snapshot is
    recovered first) and at most the persisted commit; None = the commit (a state machine that kept
    up). The committed entries above it are handed to Update again by the first tick."""
    s, R, ET = rl.state, cfg["replicas"], cfg["election_rtt"]
    last = s["last"]
    applied = s["commit"] if app_applied is None else min(max(int(app_applied), s["snap_index"]), s["commit"])
    key = (group << 32) | (slot << 24) | 1
    rto = ET + mix64(cfg["seed"] ^ mix64(key)) % ET
    match = [0] * R
    match[slot] = last
    return dict(term=s["term"], vote=s["vote"], leader=0, committed=s["commit"], applied=applied, processed=applied,
                last=last, marker=s["marker"], marker_term=s["marker_term"], snap_index=s["snap_index"],
                snap_term=s["snap_term"], cap_base=s["marker"], role=0, election_tick=0, heartbeat_tick=0,
                rand_timeout=rto, rng_ctr=1, granted=0, responded=0, active=0, err=0, drops=0,
                members=s["members"], snap_members=s["snap_members"], cc_pending=0,
                match=match, next=[last + 1] * R, rsnap=[0] * R, rstate=[0] * R)


def restore(engine, wal_logs: dict, cfg: dict, global_rids, app_applied=None):
    """Import every replica of `engine` (Engine, LoopbackCluster or Oracle: anything with
    import_replica(rid, view, terms, types, payloads, lens)) from replayed WAL logs. global_rids maps
    the engine's replica ids to global ones (identity for one rank). app_applied(global rid) -> the
    index the replica's state machine has applied (its /LastLogIndex), or None for the commit."""
    R = cfg["replicas"]
    for rid, gr in global_rids:
        rl = wal_logs[gr]
        v = restart_view(rl, gr // R, gr % R, cfg, None if app_applied is None else app_applied(gr))
        idx = range(v["marker"] + 1, v["last"] + 1)
        terms = [rl.log[i][0] for i in idx]
        # RG_ENTRY_EMPTY: an application entry whose Cmd is empty (a leader's no-op) stays empty
        types = [rl.log[i][1] | (0x100 if rl.log[i][1] == 0 and rl.log[i][2] == 0 else 0) for i in idx]
        # rg_import_replica takes the Cmds packed back to back (application entries with a Cmd only)
        pays = b"".join(rl.log[i][4] for i in idx if rl.log[i][1] == 0 and rl.log[i][2]) if cfg["payload_bytes"] else None
        lens = [rl.log[i][2] for i in idx]
        engine.import_replica(rid, v, terms, types, pays, lens)
