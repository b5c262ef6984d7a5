"""The /UpdateEntries driver (raftd_amd/apply.py) against raftd's OnDiskStateMachine.Update /
doReqWithContext (/root/reference/raft/state_machine.go:63-99, 136-166), with a local HTTP app."""
import base64
import json
import threading
from http.server import BaseHTTPRequestHandler, HTTPServer

import numpy as np
import pytest

from raftd_amd.apply import Applier, HighStatusCode, batches, parse_results, post_update, update_body
from raftd_amd.engine import APPLY_DTYPE


def fake_batch():
    recs = np.zeros(5, APPLY_DTYPE)
    rows = [(7, 3, 2, 5, 4), (8, 3, 2, 5, 4), (9, 3, 2, 3, 4), (12, 17, 1, 4, 9), (13, 17, 1, 2, 9)]
    for k, (idx, g, rep, ln, rid) in enumerate(rows):
        recs[k] = (idx, g, rep, ln, 0, rid, 16 * k)
    pay = np.zeros((5, 16), np.uint8)
    for k in range(5):
        pay[k, :recs[k]["len"]] = np.arange(recs[k]["len"]) + 10 * k
    return recs, pay


def test_batches_split_per_replica():
    bs = batches(*fake_batch())
    assert [(b.group, b.replica_id, b.rid, b.indices) for b in bs] == [(3, 2, 4, [7, 8, 9]), (17, 1, 9, [12, 13])]
    assert bs[0].cmds[2] == bytes([20, 21, 22])


def test_update_body_matches_go_encoding():
    # encoding/json of map[string]any{"Entries": []updateEntry{{5, []byte{0,1,2,3}}, {6, "hi?>"}}}
    body = update_body([5, 6], [b"\x00\x01\x02\x03", b"hi?>"])
    assert body == b'{"Entries":[{"Index":5,"Cmd":"AAECAw=="},{"Index":6,"Cmd":"aGk/Pg=="}]}'


def test_parse_results_only_when_lengths_match():
    ok = json.dumps({"Results": [{"Value": 1, "Data": base64.b64encode(b"x").decode()}, {"Value": 2, "Data": None}]})
    assert parse_results(ok.encode(), 2) == [(1, b"x"), (2, b"")]
    assert parse_results(ok.encode(), 3) is None
    assert parse_results(b'{"Result": []}', 0) is None  # README's "Result" key is ignored


class App(BaseHTTPRequestHandler):
    seen = []
    status = 200

    def do_POST(self):
        n = int(self.headers["content-length"])
        body = self.rfile.read(n)
        App.seen.append((self.path, {k.lower(): v for k, v in self.headers.items()}, body))
        if App.status != 200:
            self.send_response(App.status)
            self.end_headers()
            self.wfile.write(b"boom")
            return
        ents = json.loads(body)["Entries"]
        out = json.dumps({"Results": [{"Value": e["Index"] * 10, "Data": e["Cmd"]} for e in ents]}).encode()
        self.send_response(200)
        self.send_header("content-type", "application/json")
        self.end_headers()
        self.wfile.write(out)

    def log_message(self, *a):
        pass


@pytest.fixture
def app():
    srv = HTTPServer(("127.0.0.1", 0), App)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    App.seen, App.status = [], 200
    yield f"http://127.0.0.1:{srv.server_address[1]}"
    srv.shutdown()


class FakeEngine:
    def apply_committed(self, slot_mask=0xFF):
        return fake_batch()


def test_applier_posts_one_request_per_replica(app):
    ap = Applier(app, workers=2)
    out = ap.apply(FakeEngine())
    ap.close()
    assert len(App.seen) == 2
    by = {h["raftd-node-id"]: (p, h, b) for p, h, b in App.seen}
    p, h, b = by["3"]
    assert p == "/UpdateEntries" and h["raftd-replica-id"] == "2" and h["content-type"] == "application/json"
    assert json.loads(b)["Entries"][0] == {"Index": 7, "Cmd": base64.b64encode(bytes(range(0, 5))).decode()}
    assert out[0].results == [(70, bytes(range(0, 5))), (80, bytes(range(10, 15))), (90, bytes(range(20, 23)))]


def test_high_status_code(app):
    App.status = 500
    b = batches(*fake_batch())[0]
    with pytest.raises(HighStatusCode, match="high status code \\(500\\): boom"):
        post_update(app, b)


def test_failed_update_is_fatal(app):
    """after a failed Update the applier refuses every later batch (the device has moved
    past it; the node restarts through the WAL, which hands the batch to Update again)."""
    from raftd_amd.apply import ApplyFailed
    ap = Applier(app, workers=2)
    App.status = 500
    with pytest.raises(HighStatusCode):
        ap.apply(FakeEngine())
    App.status = 200
    n = len(App.seen)
    with pytest.raises(ApplyFailed):
        ap.apply(FakeEngine())
    assert len(App.seen) == n  # nothing posted after the failure
    ap.close()


def test_notify_after_acknowledged_updates(app):
    """notify=True reports applied = processed for the replicas of the slot mask, and only after every
    POST of the tick succeeded."""
    class Eng(FakeEngine):
        R = 3
        notified = None

        def replica_array(self):
            a = np.zeros(12, [("processed", "<u8")])
            a["processed"] = np.arange(12) + 100
            return a

        def notify_applied(self, rids, idx):
            Eng.notified = (list(rids), list(idx))

    ap = Applier(app, workers=2)
    ap.apply(Eng(), slot_mask=0b010, notify=True)
    assert Eng.notified == ([1, 4, 7, 10], [101, 104, 107, 110])
    ap.close()


def test_expand_apply_runs_with_gaps():
    """expand_apply (the host view of rg_apply_run ranges): entry k of a run is index first + k, its Cmd
    at the run's off + the 16-B-rounded lengths before it in the run; runs of several replicas."""
    from raftd_amd.engine import APPLY_CMD_DTYPE, APPLY_RUN_DTYPE, expand_apply
    cmds = np.zeros(6, APPLY_CMD_DTYPE)
    cmds["len"] = [5, 16, 17, 1, 300, 2]
    cmds["crc"] = [1, 2, 3, 4, 5, 6]
    runs = np.zeros(3, APPLY_RUN_DTYPE)
    # replica 7: indices 10, 11 then (a no-op at 12) 13; replica 9: 40, 41, 42
    runs[0] = (3, 2, 7, 10, 0, 0, 2, 0)
    runs[1] = (3, 2, 7, 13, 2, 32, 1, 0)
    runs[2] = (4, 1, 9, 40, 3, 80, 3, 0)
    out = expand_apply(runs, cmds)
    assert list(out["index"]) == [10, 11, 13, 40, 41, 42]
    assert list(out["rid"]) == [7, 7, 7, 9, 9, 9]
    assert list(out["group"]) == [3, 3, 3, 4, 4, 4]
    assert list(out["off"]) == [0, 16, 32, 80, 96, 400]
    assert list(out["len"]) == [5, 16, 17, 1, 300, 2] and list(out["crc"]) == [1, 2, 3, 4, 5, 6]
    assert len(expand_apply(np.zeros(0, APPLY_RUN_DTYPE), np.zeros(0, APPLY_CMD_DTYPE))) == 0


def test_expand_persist_ranges():
    """expand_persist (the host view of rg_persist_collect's ranges): per replica entries first..last
    at entry_off, terms from its runs, Cmds at payload_off + the rounded lengths of its earlier
    application entries (a ConfigChange's len is RG_PERSIST_CONFIG | descriptor, no Cmd bytes); a
    replica whose state changed without new entries has no rows."""
    from raftd_amd.engine import (PERSIST_CMD_DTYPE, PERSIST_CONFIG, PERSIST_STATE_DTYPE, PERSIST_TERM_DTYPE,
                                  expand_persist)
    st = np.zeros(3, PERSIST_STATE_DTYPE)
    st["rid"] = [4, 5, 6]
    st["first"], st["last"] = [20, 2**64 - 1, 7], [23, 8, 8]  # replica 5: a vote only (first > last)
    st["entry_off"], st["payload_off"], st["term_off"], st["n_terms"] = [0, 4, 4], [0, 64, 64], [0, 2, 2], [2, 0, 1]
    ents = np.zeros(6, PERSIST_CMD_DTYPE)
    ents["len"] = [5, PERSIST_CONFIG | 0x23, 0, 33, 16, 1]
    ents["crc"] = [1, 0, 0, 4, 5, 6]
    terms = np.zeros(3, PERSIST_TERM_DTYPE)
    terms["term"], terms["count"] = [3, 4, 7], [1, 3, 2]
    out = expand_persist(st, ents, terms)
    assert list(out["index"]) == [20, 21, 22, 23, 7, 8]
    assert list(out["rid"]) == [4, 4, 4, 4, 6, 6]
    assert list(out["term"]) == [3, 4, 4, 4, 7, 7]
    assert list(out["type"]) == [0, 1, 0, 0, 0, 0]
    assert list(out["len"]) == [5, 0x23, 0, 33, 16, 1]
    assert list(out["off"]) == [0, 16, 16, 16, 64, 80]
    assert len(expand_persist(st[1:2], np.zeros(0, PERSIST_CMD_DTYPE), np.zeros(0, PERSIST_TERM_DTYPE))) == 0
