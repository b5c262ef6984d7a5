"""Known-answer scenarios driven through the engine interface of tests/engines.py.

The expected values come from tests/golden/kat_*.json (published tables); these functions only
build the scenario and read back the observable result. Used by tests/test_kat.py (CPU oracles)
and tests/test_gpu_kat.py (HIP engine).
"""
from __future__ import annotations

import json
import os

import numpy as np

from engines import leader_view, log_terms, make, view

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NO_TICK = 1
RV, RV_RESP, REPL, REPL_RESP = 14, 15, 12, 13


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def small_cfg(**kw):
    c = dict(groups=1, replicas=3, log_capacity=64, payload_bytes=16, max_entries_per_msg=16)
    c.update(kw)
    return c


def run_voter(kind, case):
    e = make(kind, **small_cfg())
    e.bootstrap()
    log = case["log"]
    e.import_replica(1, view(3, term=1, last=len(log), next=[len(log) + 1] * 3), log)
    e.deliver(0, type=RV, to=2, term=3, log_term=case["cand_log_term"], log_index=case["cand_index"])
    e.tick(flags=NO_TICK)
    out = e.msgs(1, 0)
    assert len(out) == 1 and out[0]["type"] == RV_RESP and out[0]["term"] == 3, out
    return bool(out[0]["reject"])


def run_check_msgapp(kind, fix, case):
    e = make(kind, **small_cfg())
    e.bootstrap()
    log = fix["follower_log"]
    c = fix["follower_commit"]
    e.import_replica(1, view(3, term=2, leader=1, last=len(log), committed=c, applied=c,
                             next=[len(log) + 1] * 3), log)
    e.deliver(0, type=REPL, to=2, term=2, log_term=case["log_term"], log_index=case["log_index"], nent=0)
    e.tick(flags=NO_TICK)
    out = e.msgs(1, 0)
    assert len(out) == 1 and out[0]["type"] == REPL_RESP, out
    return dict(reject=bool(out[0]["reject"]), resp_index=out[0]["log_index"], hint=out[0]["hint"])


def run_append(kind, fix, case):
    e = make(kind, **small_cfg())
    e.bootstrap()
    ll = case["leader_log"]
    e.import_replica(0, leader_view(3, 0, 4, ll), ll)
    fl = fix["follower_log"]
    e.import_replica(1, view(3, term=4, leader=1, last=len(fl), next=[len(fl) + 1] * 3), fl)
    e.deliver(0, type=REPL, to=2, term=4, log_index=case["log_index"], log_term=case["log_term"],
              nent=len(case["entries"]), commit=0)
    e.tick(flags=NO_TICK)
    return log_terms(e, 1)


def run_figure7(kind, fix, ticks=80):
    followers = list(fix["followers"].values())
    R = 1 + len(followers)
    e = make(kind, **small_cfg(replicas=R))
    e.bootstrap()
    ll = fix["leader_log"] + [fix["leader_term"]]
    e.import_replica(0, leader_view(R, 0, fix["leader_term"], ll), ll)
    for k, fl in enumerate(followers):
        e.import_replica(k + 1, view(R, term=fl[-1], last=len(fl), rand_timeout=10 + k,
                                     next=[len(fl) + 1] * R), fl)
    for _ in range(ticks):
        e.tick()
    return [log_terms(e, rid) for rid in range(R)], [e.replica(rid) for rid in range(R)]


def run_current_term_commit(kind, fix):
    e = make(kind, **small_cfg())
    e.bootstrap()
    ll = fix["leader_log"] + [fix["leader_term"]]
    e.import_replica(0, leader_view(3, 0, fix["leader_term"], ll), ll)
    iso = np.array([0, 1, 1], np.uint8)
    got = []
    for ack in fix["acks"]:
        e.deliver(1, type=REPL_RESP, to=1, term=fix["leader_term"], log_index=ack["index"])
        e.tick(flags=NO_TICK, isolate=iso)
        got.append(e.replica(0)["committed"])
    return got


def run_quorum_commit(kind, case):
    n = case["size"]
    e = make(kind, **small_cfg(replicas=n))
    e.bootstrap()
    ll = [1, 2]
    v = leader_view(n, 0, 2, ll, committed=1)
    v["match"] = [1] * n + [0] * (8 - n)
    v["match"][0] = 2
    v["rstate"] = [2] * n + [0] * (8 - n)
    e.import_replica(0, v, ll)
    iso = np.array([0] + [1] * (n - 1), np.uint8)
    # one proposal entry at index 3, then acks at 3 from the acceptors
    e.tick(prop_target=np.array([0], np.uint8), prop_count=np.array([1], np.uint32), flags=NO_TICK, isolate=iso)
    for a in case["acceptors"]:
        e.deliver(a, type=REPL_RESP, to=1, term=2, log_index=3)
    e.tick(flags=NO_TICK, isolate=iso)
    return e.replica(0)["committed"] == 3
