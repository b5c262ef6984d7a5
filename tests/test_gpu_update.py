"""rg_get_update / rg_commit_update (dragonboat Peer.GetUpdate / Peer.Commit): the one
hand-off per tick must carry exactly what the four separate calls return — the persistence feed
(rg_persist_collect), the committed entries for Update (rg_apply_committed), the snapshot events
(rg_snapshot_events) and the reads made ready (rg_read_index_results) — and rg_commit_update's
applied report must move the engine exactly as rg_notify_applied does.

Two identical engines run the same chaos trace (caller Cmds of 0..300 bytes, elections, message
loss, an isolated replica that falls behind compaction and is restored by InstallSnapshot, ReadIndex
requests, apply feedback on); engine A uses the separate calls, engine B rg_get_update."""
import numpy as np
import numpy.lib.recfunctions as rfn
import pytest

from engines import make
from raftd_amd.engine import unpack_rows

pytestmark = pytest.mark.gpu


def test_get_update_equals_the_separate_calls():
    G, R, MASK = 12, 3, 0b011
    cfg = dict(groups=G, replicas=R, log_capacity=256, payload_bytes=64, max_cmd_bytes=300, max_entries_per_msg=8,
               snapshot_entries=24, compaction_overhead=3, drop_ppm=30000, apply_feedback=1, seed=0xB0B)
    a, b = make("gpu", **cfg), make("gpu", **cfg)
    for e in (a, b):
        e.bootstrap()
    rng = np.random.default_rng(11)
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    seen = {"committed": 0, "snapshots": 0, "restored": 0, "reads": 0, "states": 0}
    for t in range(90):
        iso = np.zeros(G * R, np.uint8)
        if 20 <= t < 60:
            iso[1 * R + 2] = 1  # group 1's slot 2 misses compaction, then gets InstallSnapshot
        batches = []
        if t >= 4:
            for g in range(G):
                if rng.random() < 0.7:
                    n = int(rng.integers(1, 6))
                    cmds = [bytes(rng.integers(0, 256, int(rng.integers(0, 301)), dtype=np.uint8)) for _ in range(n)]
                    batches.append((g, int(rng.integers(0, R)), cmds))
        reads = [(g, int(rng.integers(0, R)), int(rng.integers(1, 1 << 40))) for g in range(G) if rng.random() < 0.3]
        for e in (a, b):
            if batches:
                e.propose(batches)
            if t >= 4 and reads:
                e.read_index(reads)
            e.tick(campaign=camp if t == 1 else None, isolate=iso)
        st, en, rows = a.persist_collect()
        recs, arows = a.apply_committed(MASK)
        ev = a.snapshot_events(MASK)
        rd = a.read_index_results(MASK)
        u, out = b.get_update(MASK)
        assert u.tick == b.t
        # the persistence section holds the node's replicas only (slot_mask): rg_persist_collect's
        # records of those replicas, in the same order, with their own offsets
        keep = ((MASK >> (st["replica_id"].astype(np.int64) - 1)) & 1) == 1
        ekeep = ((MASK >> (en["rid"].astype(np.int64) % R)) & 1) == 1
        nooff = [f for f in st.dtype.names if f not in ("entry_off", "payload_off", "term_off")]
        assert rfn.repack_fields(out["states"][nooff]).tobytes() == rfn.repack_fields(st[keep][nooff]).tobytes(), t
        eo = [f for f in en.dtype.names if f != "off"]
        assert rfn.repack_fields(out["entries"][eo]).tobytes() == rfn.repack_fields(en[ekeep][eo]).tobytes(), t
        got = unpack_rows(out["entries"], out["entry_payload"], b.row)
        assert np.array_equal(got, rows[ekeep]), t
        assert out["committed"].tobytes() == recs.tobytes(), t
        assert np.array_equal(unpack_rows(out["committed"], out["committed_payload"], b.row), arows), t
        assert out["snapshots"].tobytes() == ev.tobytes(), t
        assert out["reads"].tobytes() == rd.tobytes(), t
        # Peer.Commit: the node's replicas applied what they were handed
        va = a.replica_array()
        rids = np.array([r for r in range(G * R) if (MASK >> (r % R)) & 1], np.uint32)
        a.notify_applied(rids, va["processed"][rids])
        b.commit_update(u, applied=True)
        assert a.replica_array().tobytes() == b.replica_array().tobytes(), t
        seen["committed"] += len(recs)
        seen["snapshots"] += int((ev["kind"] & 1).sum()) if len(ev) else 0
        seen["restored"] += int((ev["kind"] & 2).sum() != 0) if len(ev) else 0
        seen["reads"] += len(rd)
        seen["states"] += len(st)
    # the trace exercised every section
    assert all(v > 0 for v in seen.values()), seen


def test_get_update_sections_and_full_state():
    """flags select sections; RG_UPDATE_FULL_STATE = rg_persist_collect(full=1)."""
    from raftd_amd.engine import UPDATE_COMMITTED, UPDATE_FULL_STATE, UPDATE_PERSIST
    G, R = 8, 3
    e = make("gpu", groups=G, replicas=R, log_capacity=128, payload_bytes=32, max_entries_per_msg=8, seed=5)
    e.bootstrap()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    for t in range(8):
        e.tick(np.zeros(G, np.uint8) if t >= 4 else None, np.full(G, 3, np.uint32) if t >= 4 else None,
               campaign=camp if t == 1 else None)
    _, only_c = e.get_update(0xFF, UPDATE_COMMITTED)
    assert len(only_c["committed"]) > 0 and len(only_c["states"]) == 0 and len(only_c["reads"]) == 0
    _, full = e.get_update(0xFF, UPDATE_PERSIST | UPDATE_FULL_STATE)
    st, en, rows = e.persist_collect(full=True)
    assert full["states"].tobytes() == st.tobytes() and len(st) == G * R
    assert full["entries"].tobytes() == en.tobytes()
    assert np.array_equal(unpack_rows(full["entries"], full["entry_payload"], e.row), rows)
    assert len(full["committed"]) == 0


def test_get_update_against_oracle():
    """Every section of rg_get_update checked directly against the C oracle (not only against the
    engine's own separate calls): persistence records (hard state and rewritten entries with their
    Cmd bytes) of the node's replicas, committed entries per replica, snapshot events and ready reads;
    then rg_commit_update(applied) moves the engine as or_notify_applied moves the oracle."""
    G, R, MASK = 10, 3, 0b101
    cfg = dict(groups=G, replicas=R, log_capacity=128, payload_bytes=64, max_cmd_bytes=9000, max_entries_per_msg=8,
               snapshot_entries=20, compaction_overhead=3, drop_ppm=30000, apply_feedback=1, seed=0xA11,
               pool_pages=G * R * 64)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    for e in (gpu, ora):
        e.bootstrap()
    rng = np.random.default_rng(12)
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    mine = [rid for rid in range(G * R) if (MASK >> (rid % R)) & 1]
    hard = ("term", "vote", "committed", "last", "marker", "snap_index")
    prev = {rid: ora.replica(rid) for rid in mine}
    seen = dict(states=0, entries=0, committed=0, snapshots=0, reads=0)
    for t in range(70):
        iso = np.zeros(G * R, np.uint8)
        if 15 <= t < 45:
            iso[2 * R + 2] = 1  # group 2's slot 2 falls behind compaction, then InstallSnapshot
        batches = []
        if t >= 4:
            for g in range(G):
                if rng.random() < 0.6:
                    lens = rng.choice([0, 1, 64, 65, 8192, 9000, int(rng.integers(0, 9001))], int(rng.integers(1, 4)))
                    batches.append((g, int(rng.integers(0, R)),
                                    [bytes(rng.integers(0, 256, int(n), dtype=np.uint8)) for n in lens]))
        reads = [(g, int(rng.integers(0, R)), int(rng.integers(1, 1 << 40))) for g in range(G) if rng.random() < 0.3]
        for e in (gpu, ora):
            if batches:
                e.propose(batches)
            if t >= 4 and reads:
                e.read_index(reads)
            e.tick(campaign=camp if t == 1 else None, isolate=iso)
        u, out = gpu.get_update(MASK)
        # persistence: one record per node replica whose log or hard state changed, equal to the oracle
        got = {int(s["rid"]): s for s in out["states"]}
        assert set(got) <= set(mine), t
        for rid in mine:
            v = ora.replica(rid)
            if any(v[k] != prev[rid][k] for k in hard):
                assert rid in got, (t, rid)
            prev[rid] = v
        ents = out["entries"]
        for rid, s in got.items():
            v = ora.replica(rid)
            for k, f in (("term", "term"), ("vote", "vote"), ("commit", "committed"), ("last", "last"),
                         ("marker", "marker"), ("marker_term", "marker_term"), ("snap_index", "snap_index"),
                         ("snap_term", "snap_term"), ("members", "members"), ("snap_members", "snap_members")):
                assert int(s[k]) == v[f], (t, rid, k)
            first, last, lo = int(s["first"]), int(s["last"]), int(s["entry_off"])
            assert first > v["marker"]
            # the terms travel as runs: one per stretch of equal terms, strictly growing, covering first..last
            runs = out["persist_terms"][int(s["term_off"]):int(s["term_off"]) + int(s["n_terms"])]
            assert int(runs["count"].sum()) == max(0, last - first + 1), (t, rid)
            assert np.all(np.diff(runs["term"].astype(np.int64)) > 0) and np.all(runs["count"] > 0), (t, rid)
            for k, i in enumerate(range(first, last + 1)):
                pe, oe = ents[lo + k], ora.entry(rid, i, with_payload=True)
                assert (int(pe["index"]), int(pe["term"]), int(pe["type"]), int(pe["len"]), int(pe["crc"])) == \
                    (i, oe["term"], oe["type"], oe["len"], oe["crc"]), (t, rid, i)
                if oe["type"] == 0 and oe["len"]:
                    o = int(pe["off"])
                    assert bytes(out["entry_payload"][o:o + oe["len"]]) == oe["payload"], (t, rid, i)
                seen["entries"] += 1
        seen["states"] += len(got)
        # committed entries (IOnDiskStateMachine.Update input) per replica
        com = {}
        for r in out["committed"]:
            o, n = int(r["off"]), int(r["len"])
            com.setdefault(int(r["rid"]), []).append((int(r["index"]), n, int(r["crc"]),
                                                      bytes(out["committed_payload"][o:o + n])))
        for rid in range(G * R):
            assert com.get(rid, []) == (ora.applied_entries(rid) if rid in mine else []), (t, rid)
        seen["committed"] += len(out["committed"])
        # snapshot events and ready reads
        evs = {int(x["rid"]): x for x in out["snapshots"]}
        rds = {}
        for x in out["reads"]:
            rds.setdefault(int(x["rid"]), []).append((int(x["ctx"]), int(x["index"])))
        for rid in range(G * R):
            kind, restored, index, term = ora.snapshot_event(rid)
            if rid in mine and kind:
                x = evs[rid]
                assert (int(x["kind"]), int(x["restored"]), int(x["index"]), int(x["term"])) == \
                    (kind, restored, index, term), (t, rid)
            else:
                assert rid not in evs, (t, rid)
            rr = ora.read_ready(rid)
            if rid in mine and rr:
                assert rds[rid] == rr, (t, rid)
            else:
                assert rid not in rds, (t, rid)
        seen["snapshots"] += len(evs)
        seen["reads"] += len(rds)
        # Peer.Commit: the node's replicas applied what they were handed
        gpu.commit_update(u, applied=True)
        for rid in mine:
            assert ora.notify_applied(rid, ora.replica(rid)["processed"]) == 0
        for rid in range(G * R):
            assert gpu.replica(rid) == ora.replica(rid), (t, rid)
    assert all(v > 0 for v in seen.values()), seen


def test_committed_section_by_reference():
    """with the persist section in the same hand-off the committed section carries runs
    and {len, crc} only (its Cmds crossed PCIe once already, in this or an earlier persist section); the host
    resolves them from what it persisted. Two engines on one trace: A asks for the Cmds to be shipped
    (RG_UPDATE_COMMITTED_CMDS), B takes them by reference — the raw section has no payload, and the Cmds B
    resolves are A's bytes; only the persist section's Cmds crossed for B."""
    import ctypes as C
    from raftd_amd.engine import UPDATE_ALL, UPDATE_COMMITTED_CMDS, Update
    G, R, MASK = 10, 3, 0b001
    cfg = dict(groups=G, replicas=R, log_capacity=128, payload_bytes=64, max_cmd_bytes=500, max_entries_per_msg=8,
               snapshot_entries=20, compaction_overhead=3, drop_ppm=20000, seed=0xB1F)
    a, b = make("gpu", **cfg), make("gpu", **cfg)
    for e in (a, b):
        e.bootstrap()
    rng = np.random.default_rng(21)
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    shipped = resolved = 0
    for t in range(60):
        batches = []
        if t >= 4:
            for g in range(G):
                if rng.random() < 0.8:
                    cmds = [bytes(rng.integers(0, 256, int(rng.integers(0, 501)), dtype=np.uint8))
                            for _ in range(int(rng.integers(1, 5)))]
                    batches.append((g, int(rng.integers(0, R)), cmds))
        for e in (a, b):
            if batches:
                e.propose(batches)
            e.tick(campaign=camp if t == 1 else None)
        ua, oa = a.get_update(MASK, UPDATE_ALL | UPDATE_COMMITTED_CMDS)
        ub, ob = b.get_update(MASK)
        assert not oa["committed_by_reference"]
        assert oa["committed"].tobytes() == ob["committed"].tobytes(), t
        if len(ob["committed"]):
            assert ob["committed_by_reference"] and ub.committed.payload is None and ub.committed.payload_bytes == 0
            assert np.array_equal(unpack_rows(oa["committed"], oa["committed_payload"], a.row),
                                  unpack_rows(ob["committed"], ob["committed_payload"], b.row)), t
            shipped += ua.committed.payload_bytes
            resolved += len(ob["committed"])
        for e, u in ((a, ua), (b, ub)):
            e.commit_update(u, applied=True)
    assert resolved > 200 and shipped > 0
    # the raw C call: the same flags, no payload pointer, nothing but run heads and {len, crc} for the section
    u = Update()
    assert b.L.rg_get_update(b.h, MASK, UPDATE_ALL, C.byref(u)) == 0
    assert u.committed.payload_bytes == 0
