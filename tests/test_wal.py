"""Host WAL (raftd_amd/wal.py) without a GPU: record framing, torn tails, replay rules (append,
truncate-and-replace, compaction, snapshot restore) and the restart view."""
import numpy as np

from raftd_amd.engine import PERSIST_ENTRY_DTYPE, PERSIST_STATE_DTYPE
from raftd_amd.wal import WAL, records, replay, restart_view

P = 16


def rec(group, slot, term, commit, first, last, marker=0, ents=(), vote=0):
    st = np.zeros(1, PERSIST_STATE_DTYPE)
    st[0] = (group, slot + 1, 0, term, vote, commit, last, marker, term if marker else 0, marker, 0, first, 0, 7, 7, 0, 0, 0, 0)
    en = np.zeros(len(ents), PERSIST_ENTRY_DTYPE)
    pay = np.zeros((len(ents), P), np.uint8)
    for k, (i, t, ln) in enumerate(ents):
        en[k] = (i, t, 0, ln, 0, 0, k * P)
        pay[k, :ln] = (i * 7 + np.arange(ln)) & 0xFF
    return st, en, pay


def test_append_replay_truncate_compact(tmp_path):
    path = str(tmp_path / "node.wal")
    w = WAL(path)
    w.append(0, *rec(5, 1, 1, 3, 1, 3, ents=[(1, 1, 0), (2, 1, 0), (3, 1, 0)]), P)
    w.append(1, *rec(5, 1, 2, 3, 4, 8, ents=[(i, 2, P) for i in range(4, 9)]), P)
    # a conflicting leader: entries from 6 on replaced by term-3 entries, log now ends at 7
    w.append(2, *rec(5, 1, 3, 5, 6, 7, ents=[(6, 3, P), (7, 3, 0)]), P)
    # compaction to 4, no new entries (first beyond last)
    w.append(3, *rec(5, 1, 3, 7, 2 ** 64 - 1, 7, marker=4), P)
    w.close()
    logs = replay(path, replicas=3)
    rl = logs[5 * 3 + 1]
    assert rl.state["term"] == 3 and rl.state["commit"] == 7 and rl.state["marker"] == 4
    assert sorted(rl.log) == [5, 6, 7]
    assert rl.log[5][0] == 2 and rl.log[6][0] == 3 and rl.log[7][2] == 0
    assert rl.log[6][4] == bytes(((6 * 7 + np.arange(P)) & 0xFF).astype(np.uint8))


def test_torn_tail_and_corruption_are_ignored(tmp_path):
    path = str(tmp_path / "node.wal")
    w = WAL(path, sync=False)
    for t in range(3):
        w.append(t, *rec(0, 0, 1, 3, 4 + t, 4 + t, ents=[(4 + t, 1, P)]), P)
    w.close()
    data = open(path, "rb").read()
    open(path, "wb").write(data[:-10])  # crash mid-write of the last record
    assert [t for t, *_ in records(path)] == [0, 1]
    bad = bytearray(data)
    bad[60] ^= 0xFF  # corrupt the first record's body
    open(path, "wb").write(bytes(bad))
    assert list(records(path)) == []


def test_restart_view_is_a_fresh_follower():
    from raftd_amd.wal import ReplicaLog
    from oracle.pyoracle import mix64
    rl = ReplicaLog()
    rl.state = dict(term=7, vote=2, commit=40, last=44, marker=30, marker_term=6, snap_index=35, snap_term=6,
                    members=0b011, snap_members=0b111)
    cfg = dict(replicas=3, election_rtt=10, seed=0x5EED)
    v = restart_view(rl, group=9, slot=1, cfg=cfg)
    assert (v["term"], v["vote"], v["committed"], v["applied"], v["role"], v["leader"]) == (7, 2, 40, 40, 0, 0)
    assert v["match"] == [0, 44, 0] and v["next"] == [45] * 3 and v["cap_base"] == 30
    assert (v["members"], v["snap_members"], v["cc_pending"]) == (0b011, 0b111, 0)
    assert v["rand_timeout"] == 10 + mix64(0x5EED ^ mix64((9 << 32) | (1 << 24) | 1)) % 10
