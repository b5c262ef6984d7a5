"""Test helpers for the snapshot host path: the oracle behind the engine's feed interface, and a
fake raftd application (one per node) whose state per shard is a digest of the commands it
applied, so replicas that applied the same log prefix must hold the same digest."""
from __future__ import annotations

import base64
import json
import struct
import threading
import zlib
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import numpy as np

from raftd_amd.engine import APPLY_DTYPE, SNAPSHOT_EVENT_DTYPE


class OracleFeeds:
    """pyoracle.Oracle (single rank: local rid = global rid) as rg_snapshot_events /
    rg_apply_committed would hand it over."""

    def __init__(self, ora, replicas: int, payload_bytes: int):
        self.ora, self.R, self.P = ora, replicas, payload_bytes

    def _rids(self, slot_mask):
        return [rid for rid in range(self.ora.G * self.R) if (slot_mask >> (rid % self.R)) & 1]

    def snapshot_events(self, slot_mask: int = 0xFF):
        rows = []
        for rid in self._rids(slot_mask):
            kind, restored, index, term = self.ora.snapshot_event(rid)
            if kind:
                rows.append((rid // self.R, rid % self.R + 1, rid, kind, 0, restored, index, term))
        return np.array(rows, SNAPSHOT_EVENT_DTYPE)

    def apply_committed(self, slot_mask: int = 0xFF):
        recs, pays = [], []
        for rid in self._rids(slot_mask):
            for i, ln, crc, p in self.ora.applied_entries(rid):
                recs.append((i, rid // self.R, rid % self.R + 1, ln, crc, rid, len(pays) * self.P))
                pays.append(p.ljust(self.P, b"\0"))
        pay = np.frombuffer(b"".join(pays), np.uint8).reshape(len(pays), self.P) if pays else \
            np.zeros((0, self.P), np.uint8)
        return np.array(recs, APPLY_DTYPE), pay


class NodeApp:
    """A raftd application for one node: per shard {index, digest}; records every call."""

    def __init__(self):
        self.state, self.calls, self.lock = {}, [], threading.Lock()
        app = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_POST(self):
                body = self.rfile.read(int(self.headers.get("content-length") or 0))
                hdr = {k.lower(): v for k, v in self.headers.items()}
                code, out = app.handle(self.path, hdr, body)
                self.send_response(code)
                self.send_header("content-length", str(len(out)))
                self.end_headers()
                self.wfile.write(out)

        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = "http://127.0.0.1:%d" % self.srv.server_address[1]
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def handle(self, path, hdr, body):
        with self.lock:
            self.calls.append((path, hdr, body))
            if path == "/UpdateEntries":
                shard = int(hdr["raftd-node-id"])
                idx, dg = self.state.get(shard, (0, 0))
                ents = json.loads(body)["Entries"]
                for e in ents:
                    assert e["Index"] > idx, (shard, e["Index"], idx)
                    idx = e["Index"]
                    dg = zlib.crc32(struct.pack("<QI", idx, dg) + base64.b64decode(e["Cmd"]))
                self.state[shard] = (idx, dg)
                return 200, json.dumps({"Results": [{"Value": e["Index"], "Data": None} for e in ents]}).encode()
            if path == "/PrepareSnapshot":
                shard = int(hdr["raftd-node-id"])
                idx, dg = self.state.get(shard, (0, 0))
                return 200, json.dumps({"Shard": shard, "Index": idx, "Digest": dg}).encode()
            if path == "/Snapshot":
                p = json.loads(body)
                return 200, struct.pack("<QQI", int(p["Shard"]), int(p["Index"]), int(p["Digest"]))
            if path == "/RecoverFromSnapshot":
                shard, idx, dg = struct.unpack("<QQI", body)
                self.state[shard] = (idx, dg)
                return 200, b""
            return 404, b"no such endpoint in the test app"

    def close(self):
        self.srv.shutdown()
        self.srv.server_close()


def converged(apps, applied_of, groups: int, replicas: int):
    """Per group, replicas that applied up to the same index hold the same digest. Returns the
    number of (group, index) classes with more than one replica."""
    shared = 0
    for g in range(groups):
        by_applied = {}
        for s in range(replicas):
            by_applied.setdefault(applied_of(g * replicas + s), []).append(apps[s].state.get(g, (0, 0))[1])
        for a, dgs in by_applied.items():
            assert len(set(dgs)) == 1, (g, a, dgs)
            shared += len(dgs) > 1
    return shared
