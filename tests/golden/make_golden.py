"""Writes the golden fixtures under tests/golden/.

kat_*.json  — known-answer tables restated from the Raft paper and from the shapes of etcd/raft's
              paper tests (which dragonboat's raft_etcd_paper_test.go ports), as listed in
              SURVEY.md §4. Expected values are the published ones, typed in here; nothing in
              them is computed by the oracle.
crc_kat.json — CRC-32/IEEE check values (zlib-independent: computed by a bitwise loop below).
trace_*.json — per-tick digests of the C oracle on small seeded runs. These are REGRESSION
              fixtures (they pin the oracle against later edits, not against dragonboat).

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def bitwise_crc32(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0xEDB88320 if crc & 1 else 0)
    return crc ^ 0xFFFFFFFF


def bitwise_crc32c(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    return crc ^ 0xFFFFFFFF


def kats() -> dict:
    out = {}
    # etcd TestVoter shape: voter log [(term, index)], candidate (logTerm, index) → reject
    out["kat_voter.json"] = {
        "source": "etcd raft TestVoter shape (raft_paper_test.go); SURVEY.md §4 'Up-to-date rule'",
        "cases": [
            {"log": [1], "cand_log_term": 1, "cand_index": 1, "reject": False},
            {"log": [1], "cand_log_term": 1, "cand_index": 2, "reject": False},
            {"log": [1, 1], "cand_log_term": 1, "cand_index": 1, "reject": True},
            {"log": [1], "cand_log_term": 2, "cand_index": 1, "reject": False},
            {"log": [1], "cand_log_term": 2, "cand_index": 2, "reject": False},
            {"log": [1, 1], "cand_log_term": 2, "cand_index": 1, "reject": False},
            {"log": [2], "cand_log_term": 1, "cand_index": 1, "reject": True},
            {"log": [2], "cand_log_term": 1, "cand_index": 2, "reject": True},
            {"log": [2, 1], "cand_log_term": 1, "cand_index": 1, "reject": True},
        ],
    }
    # etcd TestFollowerCheckMsgApp shape: follower log [(1,1),(2,2)], commit 1
    out["kat_check_msgapp.json"] = {
        "source": "etcd raft TestFollowerCheckMsgApp shape; SURVEY.md §4 'Log matching check'",
        "follower_log": [1, 2], "follower_commit": 1,
        "cases": [
            {"log_term": 0, "log_index": 0, "reject": False, "resp_index": 1, "hint": 0},
            {"log_term": 1, "log_index": 1, "reject": False, "resp_index": 1, "hint": 0},
            {"log_term": 2, "log_index": 2, "reject": False, "resp_index": 2, "hint": 0},
            {"log_term": 1, "log_index": 2, "reject": True, "resp_index": 2, "hint": 2},
            {"log_term": 3, "log_index": 3, "reject": True, "resp_index": 3, "hint": 2},
        ],
    }
    # etcd TestFollowerAppendEntries shape: follower log [(1,1),(2,2)], commit 0
    out["kat_append.json"] = {
        "source": "etcd raft TestFollowerAppendEntries shape; SURVEY.md §4 'Truncate/append'",
        "follower_log": [1, 2],
        "cases": [
            {"log_index": 2, "log_term": 2, "entries": [3], "leader_log": [1, 2, 3], "want": [1, 2, 3]},
            {"log_index": 1, "log_term": 1, "entries": [3, 4], "leader_log": [1, 3, 4], "want": [1, 3, 4]},
            {"log_index": 0, "log_term": 0, "entries": [1], "leader_log": [1], "want": [1, 2]},
            {"log_index": 0, "log_term": 0, "entries": [3], "leader_log": [3], "want": [3]},
        ],
    }
    # Raft paper Figure 7: leader at term 8; every follower converges to the leader's log + no-op
    out["kat_figure7.json"] = {
        "source": "Ongaro & Ousterhout, 'In Search of an Understandable Consensus Algorithm', Figure 7",
        "leader_log": [1, 1, 1, 4, 4, 5, 5, 6, 6, 6],
        "leader_term": 8,
        "followers": {
            "a": [1, 1, 1, 4, 4, 5, 5, 6, 6],
            "b": [1, 1, 1, 4],
            "c": [1, 1, 1, 4, 4, 5, 5, 6, 6, 6, 6],
            "d": [1, 1, 1, 4, 4, 5, 5, 6, 6, 6, 7, 7],
            "e": [1, 1, 1, 4, 4, 4, 4],
            "f": [1, 1, 1, 2, 2, 2, 3, 3, 3, 3, 3],
        },
        "want_log": [1, 1, 1, 4, 4, 5, 5, 6, 6, 6, 8],
        "want_commit": 11,
    }
    # Figure 8 / etcd TestLeaderOnlyCommitsLogFromCurrentTerm: leader log [(1,1),(2,2)], term 3
    out["kat_current_term_commit.json"] = {
        "source": "Raft paper Figure 8 / etcd TestLeaderOnlyCommitsLogFromCurrentTerm; SURVEY.md §4",
        "leader_log": [1, 2], "leader_term": 3,
        "acks": [{"index": 1, "want_commit": 0}, {"index": 2, "want_commit": 0},
                 {"index": 3, "want_commit": 3}],
    }
    # etcd TestLeaderAcknowledgeCommit shape: every acceptor subset for sizes 1..5
    cases = []
    for n in range(1, 6):
        for mask in range(1 << (n - 1)):
            acceptors = [i + 1 for i in range(n - 1) if mask >> i & 1]  # follower slots
            cases.append({"size": n, "acceptors": acceptors,
                          "committed": len(acceptors) + 1 >= n // 2 + 1})
    out["kat_quorum_commit.json"] = {
        "source": "etcd raft TestLeaderAcknowledgeCommit shape; SURVEY.md §4 'Quorum commit'",
        "cases": cases,
    }
    # etcd TestLeaderElection: a candidate wins iff the reachable nodes (itself included) are a
    # quorum; etcd's terms start at 0, the engine's bootstrap term is 1: the campaign adds one
    out["kat_leader_election.json"] = {
        "source": "etcd raft TestLeaderElection (raft_test.go); nopStepper nodes = unreachable slots",
        "term_delta": 1,
        "cases": [
            {"size": 3, "down": [], "state": "leader"},
            {"size": 3, "down": [2], "state": "leader"},
            {"size": 3, "down": [1, 2], "state": "candidate"},
            {"size": 4, "down": [1, 2], "state": "candidate"},
            {"size": 5, "down": [1, 2], "state": "leader"},
        ],
    }
    # etcd TestCandidateFallback: a candidate that receives MsgApp from a leader of its term or a
    # higher one becomes that leader's follower at the message's term
    out["kat_candidate_fallback.json"] = {
        "source": "etcd raft TestCandidateFallback (raft_paper_test.go)",
        "cases": [{"term_delta": 0, "state": "follower"}, {"term_delta": 1, "state": "follower"}],
    }
    # etcd Test{Follower,Candidate,Leader}UpdateTermFromMessage: MsgApp at term + 1 → follower at
    # term + 1 whose leader is the sender
    out["kat_update_term.json"] = {
        "source": "etcd raft testUpdateTermFromMessage (raft_paper_test.go) for each starting state",
        "cases": [{"state": "follower"}, {"state": "candidate"}, {"state": "leader"}],
        "want_state": "follower", "want_term_delta": 1, "want_leader_is_sender": True,
    }
    # etcd TestLeaderCommitEntry: once a majority holds the new entry the leader commits it and its
    # next messages carry that commit index
    out["kat_leader_commit_entry.json"] = {
        "source": "etcd raft TestLeaderCommitEntry (raft_paper_test.go)",
        "size": 3, "leader_log": [1, 2], "leader_term": 2, "proposals": 1,
        "want_commit": 3, "want_msg_commit": 3,
    }
    # etcd TestFollowerCommitEntry: the follower commits min(leader commit, last new entry)
    out["kat_follower_commit_entry.json"] = {
        "source": "etcd raft TestFollowerCommitEntry (raft_paper_test.go)",
        "cases": [
            {"entries": [1], "commit": 1, "want_commit": 1},
            {"entries": [1, 1], "commit": 2, "want_commit": 2},
            {"entries": [1, 1], "commit": 1, "want_commit": 1},
        ],
    }
    # etcd TestVoteRequest: after its election timeout a follower campaigns at term + 1 and asks
    # every other node with its last entry's term and index
    out["kat_vote_request.json"] = {
        "source": "etcd raft TestVoteRequest (raft_paper_test.go)",
        "cases": [
            {"log": [1], "term": 1, "want_term": 2, "want_log_term": 1, "want_log_index": 1},
            {"log": [1, 2], "term": 2, "want_term": 3, "want_log_term": 2, "want_log_index": 2},
        ],
    }
    # etcd TestLeaderStepdownWhenQuorumActive / ...QuorumLost (CheckQuorum): after an election
    # timeout a leader stays only if it heard from a quorum (itself included)
    out["kat_check_quorum.json"] = {
        "source": "etcd raft TestLeaderStepdownWhenQuorumActive / TestLeaderStepdownWhenQuorumLost (raft_test.go)",
        "cases": [
            {"size": 3, "active": [], "state": "follower"},
            {"size": 3, "active": [1], "state": "leader"},
            {"size": 5, "active": [1], "state": "follower"},
            {"size": 5, "active": [1, 2], "state": "leader"},
        ],
    }
    return out


def crc_kats() -> dict:
    vecs = [b"", b"123456789", bytes(256), bytes(range(256)), b"a" * 1000]
    return {
        "source": "CRC-32/IEEE (reflected 0xEDB88320) via a bitwise loop; check value 0xCBF43926",
        "ieee": [{"hex": v.hex(), "crc": bitwise_crc32(v)} for v in vecs],
        "castagnoli_check": {"hex": b"123456789".hex(), "crc": bitwise_crc32c(b"123456789")},
    }


def trace_digest(kind_cfg: dict, ticks: int, seed: int) -> dict:
    import numpy as np
    from oracle import pyoracle as po

    o = po.Oracle(**kind_cfg)
    o.bootstrap()
    rng = np.random.default_rng(seed)
    G, R = o.G, o.R
    digests = []
    for _ in range(ticks):
        pt = rng.integers(0, R, G).astype(np.uint8)
        pt[rng.random(G) < 0.3] = 0xFF
        pc = rng.integers(1, kind_cfg["max_entries_per_msg"] + 1, G).astype(np.uint32)
        camp = (rng.random(G * R) < 0.02).astype(np.uint8)
        iso = (rng.random(G * R) < 0.05).astype(np.uint8)
        o.tick(pt, pc, camp, iso)
        h = hashlib.sha256()
        for rid in range(G * R):
            h.update(json.dumps(o.replica(rid), sort_keys=True).encode())
            for d in range(R):
                h.update(json.dumps(o.msgs(rid, d), sort_keys=True).encode())
        digests.append(h.hexdigest()[:16])
    final = [o.replica(rid) for rid in range(G * R)]
    return {"config": kind_cfg, "ticks": ticks, "input_seed": seed, "digests": digests, "final": final,
            "note": "regression fixture of the C oracle; inputs drawn with numpy default_rng(input_seed) "
                    "in the order prop_target, prop_count, campaign, isolate (see make_golden.trace_digest)"}


TRACE_CONFIGS = {
    "trace_r3_chaos.json": (dict(groups=4, replicas=3, log_capacity=64, payload_bytes=16, max_entries_per_msg=8,
                                 max_msgs_per_pair=8, num_slabs=2, election_rtt=10, heartbeat_rtt=1,
                                 check_quorum=1, snapshot_entries=20, compaction_overhead=5, drop_ppm=150000,
                                 seed=11), 150, 11),
    "trace_r5_chaos.json": (dict(groups=3, replicas=5, log_capacity=64, payload_bytes=32, max_entries_per_msg=8,
                                 max_msgs_per_pair=8, num_slabs=2, election_rtt=10, heartbeat_rtt=1,
                                 check_quorum=1, snapshot_entries=20, compaction_overhead=5, drop_ppm=150000,
                                 seed=12), 150, 12),
}


def main():
    for name, data in kats().items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(data, f, indent=1)
    with open(os.path.join(HERE, "crc_kat.json"), "w") as f:
        json.dump(crc_kats(), f, indent=1)
    for name, (cfg, ticks, seed) in TRACE_CONFIGS.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(trace_digest(cfg, ticks, seed), f)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
