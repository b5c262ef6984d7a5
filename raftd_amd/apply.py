"""raftd's apply path above the engine: committed entries → POST /UpdateEntries.

After every tick the engine copies back only what was newly committed (rg_apply_committed /
rg_apply_async: count, scan and gather kernels compact the entries each replica applied in the tick
into runs + {len, crc} + packed Cmds in device staging, and a copy kernel streams that batch into
host-mapped pinned memory; RAFTGPU_APPLY_SDMA=1 moves it with an SDMA engine instead). This module turns that
batch into the requests raftd's OnDiskStateMachine makes, byte for byte:

- ``Update`` (/root/reference/raft/state_machine.go:136-166) marshals
  ``{"Entries": [{"Index": i, "Cmd": <bytes>}]}`` with encoding/json (``[]byte`` → standard
  base64 with padding, compact separators, fields in declaration order) and takes the response's
  ``Results`` (``[]statemachine.Result{Value uint64, Data []byte}``) only when its length equals
  the number of entries (:158-163);
- ``doReqWithContext`` (:63-99) POSTs with headers ``raftd-node-id`` = the shard id and
  ``raftd-replica-id`` = the replica id, ``content-type: application/json``, a 1 s timeout
  (:47), and fails with "high status code" above 299 (:54-61).

One request per (shard, replica) and tick, as dragonboat hands a replica's applied batch to one
Update call. Requests for different replicas are independent (dragonboat serialises Update per
shard only) and go out concurrently.
"""
from __future__ import annotations

import base64
import json
import urllib.error
import urllib.request
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

TIMEOUT_S = 1.0  # raft/state_machine.go:47 `timeout = time.Second`
JSON_CONTENT_TYPE = "application/json"


class HighStatusCode(RuntimeError):
    """raft/state_machine.go:44 ErrHighStatusCode."""

    def __init__(self, status: int, body: bytes):
        super().__init__(f"high status code ({status}): {body[:100].decode(errors='replace')}")
        self.status = status


@dataclass
class UpdateBatch:
    """The entries one replica applied in one tick (one Update call)."""
    group: int         # shard id → raftd-node-id
    replica_id: int    # → raftd-replica-id
    rid: int           # local replica id in the engine
    indices: list = field(default_factory=list)
    cmds: list = field(default_factory=list)
    results: list | None = None  # [(Value, Data)] when the application answered with one per entry


def batches(recs, pay) -> list:
    """Split an rg_apply_committed batch (grouped by replica, each in index order) per replica."""
    out, cur = [], None
    for k in range(len(recs)):
        r = recs[k]
        rid = int(r["rid"])
        if cur is None or cur.rid != rid:
            cur = UpdateBatch(group=int(r["group"]), replica_id=int(r["replica_id"]), rid=rid)
            out.append(cur)
        cur.indices.append(int(r["index"]))
        cur.cmds.append(bytes(pay[k, :int(r["len"])]))
    return out


def update_body(indices, cmds) -> bytes:
    """json.Marshal(map[string]any{"Entries": []updateEntry{{Index, Cmd}}}) as Go writes it."""
    ents = [{"Index": int(i), "Cmd": base64.b64encode(c).decode("ascii")} for i, c in zip(indices, cmds)]
    return json.dumps({"Entries": ents}, separators=(",", ":")).encode()


def parse_results(body: bytes, n: int):
    """updateResponse{Results []statemachine.Result}: [(Value, Data)] if there is one per entry."""
    d = json.loads(body)
    res = d.get("Results") if isinstance(d, dict) else None
    if not isinstance(res, list) or len(res) != n:
        return None
    out = []
    for x in res:
        data = x.get("Data")
        out.append((int(x.get("Value", 0)), base64.b64decode(data) if data else b""))
    return out


def post_update(app_url: str, b: UpdateBatch, timeout: float = TIMEOUT_S) -> UpdateBatch:
    req = urllib.request.Request(app_url + "/UpdateEntries", data=update_body(b.indices, b.cmds), method="POST")
    req.add_header("raftd-node-id", str(b.group))
    req.add_header("raftd-replica-id", str(b.replica_id))
    req.add_header("content-type", JSON_CONTENT_TYPE)
    try:
        with urllib.request.urlopen(req, timeout=timeout) as resp:
            body = resp.read()
    except urllib.error.HTTPError as e:
        raise HighStatusCode(e.code, e.read()) from None
    b.results = parse_results(body, len(b.indices))
    return b


class ApplyFailed(RuntimeError):
    """An Update failed earlier: the node must restart (dragonboat stops a node whose state machine
    Update returns an error); further batches are refused so none is silently skipped."""


class Applier:
    """Drives /UpdateEntries from the engine's committed-entry copy-back after each tick.

    Failure contract: the first failed POST (timeout, transport error, status > 299) is
    fatal — apply() re-raises it and every later call raises ApplyFailed, because the device has
    already moved past that batch. The node restarts through the WAL path: with
    rg_config.apply_feedback = 1 and notify=True the engine's `applied` only ever moved for batches
    the application acknowledged, the restart view starts from the app's /LastLogIndex, and the
    first tick hands the unacknowledged entries to Update again (raftd_amd/wal.py restart_view)."""

    def __init__(self, app_url: str, workers: int = 16, timeout: float = TIMEOUT_S):
        self.app_url = app_url.rstrip("/")
        self.timeout = timeout
        self.pool = ThreadPoolExecutor(max_workers=workers)
        self.failed = None

    def apply(self, engine, slot_mask: int = 0xFF, notify: bool = False) -> list:
        """POST the last tick's applied entries of the replicas in slot_mask (one request per
        replica). notify: once every POST succeeded, report applied = processed for those replicas
        (rg_notify_applied; config changes and empty entries included — the state machine never
        sees them, dragonboat's rsm applies them itself)."""
        if self.failed is not None:
            raise ApplyFailed(f"an earlier Update failed ({self.failed}); restart the node from its WAL")
        recs, pay = engine.apply_committed(slot_mask)
        bs = batches(recs, pay)
        try:
            out = list(self.pool.map(lambda b: post_update(self.app_url, b, self.timeout), bs))
        except Exception as ex:
            self.failed = ex
            raise
        if notify:
            import numpy as np
            va = engine.replica_array()
            rids = np.array([r for r in range(len(va)) if (slot_mask >> (r % engine.R)) & 1], np.uint32)
            if len(rids):
                engine.notify_applied(rids, va["processed"][rids])
        return out

    def close(self):
        self.pool.shutdown(wait=True)
