"""Snapshot host path: the state-machine calls around the engine's snapshots.

The engine decides snapshots on the device: at the end of a tick a replica with
SnapshotEntries applied since its last snapshot records one at ``applied`` and compacts its log to
``applied - CompactionOverhead``; a follower whose ``next`` fell below its leader's compaction
marker receives InstallSnapshot and restores its log to the snapshot's index. dragonboat's rsm
turns those into calls on raftd's ``OnDiskStateMachine``, which forwards each to the application:

- ``PrepareSnapshot`` (/root/reference/raft/state_machine.go:186-197): ``doReqWithContext[any]``
  POST ``/PrepareSnapshot`` with the ``raftd-node-id`` / ``raftd-replica-id`` headers, no body,
  no content-type, 1 s timeout, the response JSON-decoded into ``any``;
- ``SaveSnapshot`` (:199-232): POST ``/Snapshot`` with ``json.Marshal`` of that value,
  ``content-type: application/json``, NO raftd headers, 1 min timeout; the raw response body is
  the snapshot data (``io.Copy`` into dragonboat's snapshot writer);
- ``RecoverFromSnapshot`` (:234-256): POST ``/RecoverFromSnapshot`` with the snapshot bytes,
  ``content-type: application/octet-stream``, NO raftd headers, 1 min timeout.

Any status above 299 fails with "high status code" (:54-61). (The reference formats that error
with ``string(body)[:100]``, which panics on bodies shorter than 100 bytes; here the message is
truncated instead.)

``rg_snapshot_events`` hands over, per tick, every replica that restored (``restored``) or took a
snapshot (``index``, ``term``). ``SnapshotDriver.after_tick`` runs, per replica and in
dragonboat's order, RecoverFromSnapshot (the snapshot the leader saved at ``restored``; the
replica keeps a copy, as dragonboat's follower keeps the received file), the tick's Update batch
(entries above the restored index, raftd_amd/apply.py), then PrepareSnapshot + SaveSnapshot into
the ``SnapshotStore``. Replicas run concurrently, each replica's calls in order
(dragonboat serialises them per shard replica).

The store keeps each replica's snapshots as fsynced files (``<dir>/<group>/<replica>/<index>``:
header + data + CRC-32), the newest ``keep`` per replica: an InstallSnapshot is delivered one tick
after its leader sent it, and the leader takes at most one newer snapshot in between, so keep=2
always holds the one being restored (all restores of a tick fetch before any save of that tick).
In raftd the follower's NodeHost receives that file from the leader's over dragonboat's
transport before the message is delivered; moving snapshot files
between hosts is transport work (out of scope), so the driver takes a ``fetch``
callable and defaults to the local store, which serves every replica hosted by this process.
"""
from __future__ import annotations

import json
import math
import os
import struct
import urllib.error
import urllib.request
import zlib
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from decimal import Decimal

from .apply import JSON_CONTENT_TYPE, TIMEOUT_S, HighStatusCode, UpdateBatch, batches, post_update
from .engine import SNAP_RESTORED, SNAP_TAKEN

SNAPSHOT_TIMEOUT_S = 60.0  # raft/state_machine.go:48 `snapshotTimeout = time.Minute`
BYTES_CONTENT_TYPE = "application/octet-stream"  # :50


# ------------------------------------------------------------------ Go encoding/json of `any`

def _go_float(f: float) -> str:
    """encoding/json floatEncoder (64-bit): shortest round-trip digits, fixed notation unless
    |f| < 1e-6 or |f| >= 1e21, exponent without a leading zero (e-07 → e-7)."""
    if math.isnan(f) or math.isinf(f):
        raise ValueError(f"json: unsupported value: {f}")
    a = abs(f)
    if a != 0 and (a < 1e-6 or a >= 1e21):
        s = repr(f)
        if "e" not in s:  # repr prints some small values in fixed notation
            s = "%.17g" % f
            s = repr(float(s)) if "e" in repr(float(s)) else s
        m, e = s.split("e")
        if "." in m:
            m = m.rstrip("0").rstrip(".")
        sign, digits = e[0], e[1:].lstrip("0") or "0"
        return f"{m}e{sign}{digits.zfill(2) if sign == '+' else digits}"
    if f == 0:
        return "-0" if math.copysign(1.0, f) < 0 else "0"
    s = format(Decimal(repr(f)), "f")
    if "." in s:
        s = s.rstrip("0").rstrip(".")
    return s


def _go_string(s: str) -> str:
    """encoding/json string encoder with HTML escaping (json.Marshal's default); invalid UTF-16
    surrogates become U+FFFD as Go's decoder leaves them."""
    out = ['"']
    for ch in s:
        c = ord(ch)
        if 0xD800 <= c <= 0xDFFF:
            out.append("�")
        elif ch in '\\"':
            out.append("\\" + ch)
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif ch == "\b":
            out.append("\\b")
        elif ch == "\f":
            out.append("\\f")
        elif c < 0x20 or ch in "<>&" or c in (0x2028, 0x2029):
            out.append("\\u%04x" % c)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def go_marshal(v) -> bytes:
    """json.Marshal of a value json.Unmarshal decoded into `any`: objects with keys sorted,
    every number a float64, compact."""
    def enc(x):
        if x is None:
            return "null"
        if x is True:
            return "true"
        if x is False:
            return "false"
        if isinstance(x, (int, float)):
            return _go_float(float(x))
        if isinstance(x, str):
            return _go_string(x)
        if isinstance(x, list):
            return "[" + ",".join(enc(y) for y in x) + "]"
        if isinstance(x, dict):
            return "{" + ",".join(_go_string(k) + ":" + enc(x[k]) for k in sorted(x)) + "}"
        raise TypeError(f"json: unsupported type: {type(x).__name__}")
    return enc(v).encode("utf-8", "surrogatepass")


def go_unmarshal_any(body: bytes):
    """json.Unmarshal into `any`: numbers are float64 (out of range → error)."""
    def num(s):
        f = float(s)
        if math.isinf(f):
            raise ValueError(f"json: cannot unmarshal number {s} into Go value of type float64")
        return f
    return json.loads(body.decode("utf-8", "replace"), parse_int=num, parse_float=num)


# ------------------------------------------------------------------ the three application calls

def _post(req, timeout):
    try:
        with urllib.request.urlopen(req, timeout=timeout) as resp:
            return resp.read()
    except urllib.error.HTTPError as e:
        raise HighStatusCode(e.code, e.read()) from None


def prepare_snapshot(app_url: str, group: int, replica_id: int, timeout: float = TIMEOUT_S):
    """OnDiskStateMachine.PrepareSnapshot: the application's JSON answer, decoded as Go does."""
    # nil body, no content-type: urllib then sends Content-Length: 0 and no Content-Type, as Go
    req = urllib.request.Request(app_url + "/PrepareSnapshot", data=None, method="POST")
    req.add_header("raftd-node-id", str(group))
    req.add_header("raftd-replica-id", str(replica_id))
    return go_unmarshal_any(_post(req, timeout))


def save_snapshot(app_url: str, prepared, timeout: float = SNAPSHOT_TIMEOUT_S) -> bytes:
    """OnDiskStateMachine.SaveSnapshot: the snapshot data the application streams back."""
    req = urllib.request.Request(app_url + "/Snapshot", data=go_marshal(prepared), method="POST")
    req.add_header("content-type", JSON_CONTENT_TYPE)
    return _post(req, timeout)


def recover_from_snapshot(app_url: str, data: bytes, timeout: float = SNAPSHOT_TIMEOUT_S) -> None:
    """OnDiskStateMachine.RecoverFromSnapshot."""
    req = urllib.request.Request(app_url + "/RecoverFromSnapshot", data=bytes(data), method="POST")
    req.add_header("content-type", BYTES_CONTENT_TYPE)
    _post(req, timeout)


# ------------------------------------------------------------------ durable snapshot files

SNAP_MAGIC = b"RGSN"
SNAP_HDR = struct.Struct("<4sIQIIQQQI")  # magic, version, group, replica_id, pad, index, term, len, crc


class SnapshotStore:
    """Snapshot files per replica, written atomically (temp file, fsync, rename, fsync dir)."""

    def __init__(self, root: str, keep: int = 2, sync: bool = True):
        self.root, self.keep, self.sync = root, keep, sync
        os.makedirs(root, exist_ok=True)

    def _dir(self, group: int, replica_id: int) -> str:
        return os.path.join(self.root, "%016x" % group, str(replica_id))

    def save(self, group: int, replica_id: int, index: int, term: int, data: bytes) -> str:
        d = self._dir(group, replica_id)
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, "%016x" % index)
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(SNAP_HDR.pack(SNAP_MAGIC, 1, group, replica_id, 0, index, term, len(data), zlib.crc32(data)))
            f.write(data)
            f.flush()
            if self.sync:
                os.fsync(f.fileno())
        os.replace(tmp, path)
        if self.sync:
            fd = os.open(d, os.O_RDONLY)
            try:
                os.fsync(fd)
            finally:
                os.close(fd)
        for old in self.indices(group, replica_id)[:-self.keep]:
            os.remove(os.path.join(d, "%016x" % old))
        return path

    def indices(self, group: int, replica_id: int) -> list:
        d = self._dir(group, replica_id)
        if not os.path.isdir(d):
            return []
        return sorted(int(n, 16) for n in os.listdir(d) if not n.endswith(".tmp"))

    def load(self, group: int, replica_id: int, index: int):
        """(term, data) of a stored snapshot; ValueError if the file is damaged."""
        with open(os.path.join(self._dir(group, replica_id), "%016x" % index), "rb") as f:
            raw = f.read()
        if len(raw) < SNAP_HDR.size:
            raise ValueError("snapshot file truncated")
        magic, ver, g, rep, _, idx, term, n, crc = SNAP_HDR.unpack_from(raw)
        data = raw[SNAP_HDR.size:]
        if magic != SNAP_MAGIC or ver != 1 or (g, rep, idx) != (group, replica_id, index) or len(data) != n \
                or zlib.crc32(data) != crc:
            raise ValueError("snapshot file damaged")
        return term, data

    def find(self, group: int, index: int, replicas: int):
        """(term, data) of any replica's snapshot of `group` at `index` (None if none holds one):
        replicas that applied the same committed log hold the same state at the same index."""
        for rep in range(1, replicas + 1):
            if index in self.indices(group, rep):
                return self.load(group, rep, index)
        return None


# ------------------------------------------------------------------ the per-tick driver

@dataclass
class ReplicaTick:
    """What one replica handed to its state machine in one tick, in call order."""
    group: int
    replica_id: int
    rid: int
    restored: int = 0                 # RecoverFromSnapshot at this index (0: none)
    update: UpdateBatch | None = None  # Update of the tick's applied entries
    snapshot: tuple | None = None      # (index, term) saved after the Update
    restore_data: tuple | None = None  # (term, data) of the snapshot at `restored`
    calls: list = field(default_factory=list)


class SnapshotDriver:
    """After each tick: snapshot restores, the /UpdateEntries batch and snapshot saves, per replica
    in dragonboat's order. `engine` is anything with snapshot_events() and apply_committed().

    app_url: the application's URL, or {replica_id: URL} when this process hosts replicas of
    several raftd nodes (each node talks to its own application, env.ApplicationURL; Recover and
    Snapshot requests carry no replica header, so one application cannot serve two replicas of a
    shard)."""

    def __init__(self, app_url, store: SnapshotStore, replicas: int, fetch=None, workers: int = 16,
                 timeout: float = TIMEOUT_S, snapshot_timeout: float = SNAPSHOT_TIMEOUT_S):
        urls = app_url if isinstance(app_url, dict) else {r: app_url for r in range(1, replicas + 1)}
        self.urls = {int(r): u.rstrip("/") for r, u in urls.items()}
        self.store, self.replicas = store, replicas
        self.fetch = fetch or (lambda group, index: self.store.find(group, index, self.replicas))
        self.timeout, self.snapshot_timeout = timeout, snapshot_timeout
        self.pool = ThreadPoolExecutor(max_workers=workers)

    def plan(self, events, recs, pay) -> list:
        """ReplicaTick per replica with anything to do, by replica id."""
        per = {}
        for ev in events:
            rt = per.setdefault(int(ev["rid"]), ReplicaTick(int(ev["group"]), int(ev["replica_id"]), int(ev["rid"])))
            if int(ev["kind"]) & SNAP_RESTORED:
                rt.restored = int(ev["restored"])
            if int(ev["kind"]) & SNAP_TAKEN:
                rt.snapshot = (int(ev["index"]), int(ev["term"]))
        for b in batches(recs, pay):
            rt = per.setdefault(b.rid, ReplicaTick(b.group, b.replica_id, b.rid))
            rt.update = b
        return [per[k] for k in sorted(per)]

    def run_replica(self, rt: ReplicaTick) -> ReplicaTick:
        url = self.urls[rt.replica_id]
        if rt.restored:
            term, data = rt.restore_data
            recover_from_snapshot(url, data, self.snapshot_timeout)
            # the replica keeps the received snapshot (it may serve it as leader later)
            self.store.save(rt.group, rt.replica_id, rt.restored, term, data)
            rt.calls.append(("RecoverFromSnapshot", rt.restored))
        if rt.update is not None:
            post_update(url, rt.update, self.timeout)
            rt.calls.append(("Update", rt.update.indices[0], rt.update.indices[-1]))
        if rt.snapshot is not None:
            prepared = prepare_snapshot(url, rt.group, rt.replica_id, self.timeout)
            data = save_snapshot(url, prepared, self.snapshot_timeout)
            self.store.save(rt.group, rt.replica_id, rt.snapshot[0], rt.snapshot[1], data)
            rt.calls.append(("SaveSnapshot", rt.snapshot[0]))
        return rt

    def after_tick(self, engine, slot_mask: int = 0xFF) -> list:
        events = engine.snapshot_events(slot_mask)
        recs, pay = engine.apply_committed(slot_mask)
        work = self.plan(events, recs, pay)
        # a restore reads a snapshot saved in an earlier tick; fetch them all before any save of
        # this tick can prune one
        for rt in work:
            if rt.restored:
                rt.restore_data = self.fetch(rt.group, rt.restored)
                if rt.restore_data is None:
                    raise LookupError(f"no snapshot of shard {rt.group} at index {rt.restored}")
        return list(self.pool.map(self.run_replica, work))

    def close(self):
        self.pool.shutdown(wait=True)
