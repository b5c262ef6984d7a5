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


# ---- etcd raft paper-test shapes (tests/golden/kat_*.json; parity with dragonboat unpinned)
ROLES = {0: "follower", 1: "candidate", 2: "leader"}
HB_RESP = 18


def _booted(kind, n, **kw):
    e = make(kind, **small_cfg(replicas=n, **kw))
    e.bootstrap()
    e.tick(flags=NO_TICK)  # the bootstrap entries are applied: campaigns are allowed
    return e


def run_leader_election(kind, case):
    """etcd TestLeaderElection: slot 0 campaigns; `down` slots are unreachable."""
    n = case["size"]
    e = _booted(kind, n)
    iso = np.zeros(n, np.uint8)
    iso[case["down"]] = 1
    t0 = e.replica(0)["term"]
    camp = np.zeros(n, np.uint8)
    camp[0] = 1
    e.tick(campaign=camp, isolate=iso, flags=NO_TICK)
    for _ in range(3):
        e.tick(isolate=iso, flags=NO_TICK)
    v = e.replica(0)
    return ROLES[v["role"]], v["term"] - t0


def run_candidate_fallback(kind, case):
    """etcd TestCandidateFallback: a candidate receives MsgApp at its term (+ delta) from slot 1."""
    e = _booted(kind, 3)
    iso = np.array([0, 1, 1], np.uint8)
    e.tick(campaign=np.array([1, 0, 0], np.uint8), isolate=iso, flags=NO_TICK)
    t = e.replica(0)["term"]
    assert e.replica(0)["role"] == 1
    e.deliver(1, type=REPL, to=1, term=t + case["term_delta"], log_index=0, log_term=0, nent=0)
    e.tick(isolate=iso, flags=NO_TICK)
    v = e.replica(0)
    return ROLES[v["role"]], v["term"] - t, v["leader"]


def run_update_term(kind, case):
    """etcd testUpdateTermFromMessage: slot 0 as follower / candidate / leader receives MsgApp at
    term + 1 from slot 1."""
    e = _booted(kind, 3)
    if case["state"] != "follower":
        iso = np.array([0, 1, 1], np.uint8) if case["state"] == "candidate" else None
        e.tick(campaign=np.array([1, 0, 0], np.uint8), isolate=iso, flags=NO_TICK)
        for _ in range(3 if case["state"] == "leader" else 0):
            e.tick(flags=NO_TICK)
    v0 = e.replica(0)
    assert ROLES[v0["role"]] == case["state"], v0
    iso = np.array([0, 1, 1], np.uint8)
    e.deliver(1, type=REPL, to=1, term=v0["term"] + 1, log_index=0, log_term=0, nent=0)
    e.tick(isolate=iso, flags=NO_TICK)
    v = e.replica(0)
    return ROLES[v["role"]], v["term"] - v0["term"], v["leader"]


def run_leader_commit_entry(kind, fix):
    """etcd TestLeaderCommitEntry: the leader commits its proposal once a majority holds it and
    its next messages carry the new commit index."""
    n, ll, t = fix["size"], fix["leader_log"], fix["leader_term"]
    e = make(kind, **small_cfg(replicas=n))
    e.bootstrap()
    e.import_replica(0, leader_view(n, 0, t, ll, committed=len(ll)), ll)
    for k in range(1, n):
        e.import_replica(k, view(n, term=t, leader=1, last=len(ll), committed=len(ll), applied=len(ll),
                                 next=[len(ll) + 1] * n), ll)
    e.tick(prop_target=np.array([0], np.uint8), prop_count=np.array([fix["proposals"]], np.uint32), flags=NO_TICK)
    msg_commit = None
    for _ in range(6):
        e.tick(flags=NO_TICK)
        if e.replica(0)["committed"] == fix["want_commit"]:
            msg_commit = max(m["commit"] for d in range(1, n) for m in e.msgs(0, d))
            break
    return e.replica(0)["committed"], msg_commit


def run_follower_commit_entry(kind, case):
    """etcd TestFollowerCommitEntry: an empty follower receives MsgApp with the entries and a commit."""
    ents = case["entries"]
    e = make(kind, **small_cfg())
    e.bootstrap()
    e.import_replica(0, leader_view(3, 0, 1, ents, committed=0), ents)
    e.import_replica(1, view(3, term=1, leader=1, last=0, next=[1] * 3), [])
    e.deliver(0, type=REPL, to=2, term=1, log_index=0, log_term=0, nent=len(ents), commit=case["commit"])
    e.tick(isolate=np.array([1, 0, 1], np.uint8), flags=NO_TICK)
    return e.replica(1)["committed"]


def run_vote_request(kind, case):
    """etcd TestVoteRequest: a follower with `log` at `term` campaigns and asks every other node."""
    log = case["log"]
    e = make(kind, **small_cfg())
    e.bootstrap()
    e.import_replica(0, view(3, term=case["term"], last=len(log), next=[len(log) + 1] * 3), log)
    e.tick(campaign=np.array([1, 0, 0], np.uint8), flags=NO_TICK)
    out = []
    for d in (1, 2):
        ms = [m for m in e.msgs(0, d) if m["type"] == RV]
        assert len(ms) == 1, ms
        out.append((ms[0]["term"], ms[0]["log_term"], ms[0]["log_index"]))
    return out


def run_check_quorum(kind, case):
    """etcd TestLeaderStepdownWhenQuorum{Active,Lost}: a fresh leader hears only from `active`
    slots (HeartbeatResp every tick) for an election timeout + 1 ticks."""
    n = case["size"]
    e = make(kind, **small_cfg(replicas=n, check_quorum=1, election_rtt=10))
    e.bootstrap()
    ll = [1] * n + [2]
    e.import_replica(0, leader_view(n, 0, 2, ll, committed=n), ll)
    iso = np.array([0] + [1] * (n - 1), np.uint8)
    for _ in range(10 + 1):
        for a in case["active"]:
            e.deliver(a, type=HB_RESP, to=1, term=2)
        e.tick(isolate=iso)
    return ROLES[e.replica(0)["role"]]


def _paper_kats():
    """name → check(kind) returning one bool per case, for the etcd paper-test shapes above."""
    def election(k):
        f = load("kat_leader_election.json")
        return [run_leader_election(k, c) == (c["state"], f["term_delta"]) for c in f["cases"]]

    def fallback(k):
        return [run_candidate_fallback(k, c) == (c["state"], c["term_delta"], 2)
                for c in load("kat_candidate_fallback.json")["cases"]]

    def update_term(k):
        f = load("kat_update_term.json")
        return [run_update_term(k, c) == (f["want_state"], f["want_term_delta"], 2) for c in f["cases"]]

    def leader_commit(k):
        f = load("kat_leader_commit_entry.json")
        return [run_leader_commit_entry(k, f) == (f["want_commit"], f["want_msg_commit"])]

    def follower_commit(k):
        return [run_follower_commit_entry(k, c) == c["want_commit"]
                for c in load("kat_follower_commit_entry.json")["cases"]]

    def vote_request(k):
        return [run_vote_request(k, c) == [(c["want_term"], c["want_log_term"], c["want_log_index"])] * 2
                for c in load("kat_vote_request.json")["cases"]]

    def check_quorum(k):
        return [run_check_quorum(k, c) == c["state"] for c in load("kat_check_quorum.json")["cases"]]

    return dict(leader_election=election, candidate_fallback=fallback, update_term=update_term,
                leader_commit_entry=leader_commit, follower_commit_entry=follower_commit,
                vote_request=vote_request, check_quorum=check_quorum)


PAPER_KATS = _paper_kats()


# ---- the engine's own boundary (not a published table): terms are 36-bit
TERM_MAX = (1 << 36) - 1
ERR_TERM_LIMIT = 128


def run_term_limit(kind, term):
    """A follower at `term` campaigns: below the limit it becomes a candidate at term + 1 and asks
    for votes; at 2^36 - 1 the campaign is refused (RG_ERR_TERM_LIMIT), the replica stays a follower
    at its term and sends nothing."""
    e = make(kind, **small_cfg())
    e.bootstrap()
    log = [1, 1, 1]
    e.import_replica(0, view(3, term=term, last=3, committed=3, applied=3, next=[4] * 3), log)
    e.tick(campaign=np.array([1, 0, 0], np.uint8), flags=NO_TICK)
    v = e.replica(0)
    sent = sum(len([m for m in e.msgs(0, d) if m["type"] == RV]) for d in (1, 2))
    return ROLES[v["role"]], v["term"], v["err"], sent
