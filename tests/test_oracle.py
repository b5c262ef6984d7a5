"""The C oracle against its pins: CRC check values, the independent Python restatement
(tick-by-tick on random chaotic traces), and the committed regression traces."""
import hashlib
import json

import numpy as np
import pytest

import kat_scenarios as K
from engines import make
from oracle import pyoracle, pyraft


def test_crc_kats():
    d = K.load("crc_kat.json")
    for v in d["ieee"]:
        assert pyoracle.crc32(bytes.fromhex(v["hex"])) == v["crc"]
    assert pyoracle.crc32(b"123456789") == 0xCBF43926
    c = d["castagnoli_check"]
    assert pyoracle.crc32c(bytes.fromhex(c["hex"])) == c["crc"] == 0xE3069283


def test_crc32c_matches_bitwise_restatement():
    from test_gpu_parity import crc32c_py
    rng = np.random.default_rng(3)
    for n in (0, 1, 15, 16, 255, 256, 1024):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert pyoracle.crc32c(b) == crc32c_py(b)


def test_oracle_entry_crcs_follow_config():
    from test_gpu_parity import crc32c_py
    import zlib
    for c32c in (0, 1):
        o = pyoracle.Oracle(groups=2, replicas=3, payload_bytes=64, max_entries_per_msg=8, crc32c=c32c)
        o.bootstrap()
        o.tick()  # the bootstrap ConfigChange entries apply first; a campaign before that is dropped
        o.tick(campaign=np.array([1, 0, 0, 1, 0, 0], np.uint8))
        for _ in range(12):
            o.tick(np.zeros(2, np.uint8), np.full(2, 3, np.uint32))
        v = o.replica(1)
        assert v["last"] >= 12, v
        for i in range(v["marker"] + 1, v["last"] + 1):
            e = o.entry(1, i, with_payload=True)
            if e["len"] and e["type"] == 0:  # ConfigChange entries carry a descriptor in len, no Cmd
                assert e["crc"] == (crc32c_py(e["payload"]) if c32c else zlib.crc32(e["payload"]))


def test_mix64_and_payload_agree():
    o = pyoracle.Oracle(groups=2, replicas=3, payload_bytes=64)
    for z in (0, 1, 0x5EED, 2**63 + 12345):
        assert pyoracle.mix64(z) == pyraft.mix64(z)
    for sl, g, i in ((0, 0, 0), (1, 1, 63), (1, 0, 5)):
        assert o.payload(sl, g, i) == pyraft.payload(0x5EED, sl, g, i, 64)


def random_inputs(rng, G, R, emax):
    pt = rng.integers(0, R, G).astype(np.uint8)
    pt[rng.random(G) < 0.3] = 0xFF
    pc = rng.integers(1, emax + 1, G).astype(np.uint32)
    camp = (rng.random(G * R) < 0.02).astype(np.uint8)
    iso = (rng.random(G * R) < 0.05).astype(np.uint8)
    return pt, pc, camp, iso


def cross_check(seed, G, R, T, **cfg):
    kw = dict(groups=G, replicas=R, payload_bytes=16, max_entries_per_msg=8, log_capacity=64,
              snapshot_entries=20, compaction_overhead=5, drop_ppm=150000, seed=seed)
    kw.update(cfg)
    a, b = make("c", **kw), make("py", **kw)
    a.bootstrap()
    b.bootstrap()
    rng = np.random.default_rng(seed)
    for t in range(T):
        ins = random_inputs(rng, G, R, kw["max_entries_per_msg"])
        a.tick(*ins)
        b.tick(*ins)
        for rid in range(G * R):
            va = a.replica(rid)
            assert va == b.replica(rid), (seed, t, rid)
            for d in range(R):
                assert a.msgs(rid, d) == b.msgs(rid, d), (seed, t, rid, d)
            for i in range(va["marker"] + 1, va["last"] + 1):
                assert a.entry(rid, i) == b.entry(rid, i), (seed, t, rid, i)


def random_batches(rng, G, R, E, P, base=0, p_none=0.3, maxc=None):
    """Caller proposals for one tick: per group (with probability 1 - p_none) a batch of 1..E Cmds
    to a random slot, lengths drawn from the edge cases 0, 1, 17, P and uniform [0, P]; with
    maxc > P (max_cmd_bytes) also P - 1, P + 1, maxc and uniform [0, maxc]."""
    M = maxc or P
    out = []
    for g in range(G):
        if rng.random() < p_none:
            continue
        n = int(rng.integers(1, E + 1))
        pool = [0, 1, min(17, P), P, int(rng.integers(0, P + 1))]
        if M > P:
            pool += [P - 1, P + 1, M, int(rng.integers(0, M + 1)), int(rng.integers(P, M + 1))]
        lens = [int(x) for x in rng.choice(pool, n)]
        cmds = [rng.integers(0, 256, ln, dtype=np.uint8).tobytes() for ln in lens]
        out.append((base + g, int(rng.integers(0, R)), cmds))
    return out


BIG_LENS = (8191, 8192, 65536, 1 << 20)  # the old 13-bit length field's edge, one past it, 64 KiB, 1 MiB


def big_batches(rng, G, R, P, base=0, p_none=0.4, nmax=3):
    """Caller proposals with Cmds far longer than payload_bytes: per group (probability 1 - p_none)
    1..nmax Cmds whose lengths come from BIG_LENS, the small edge cases (0, 1, P) and uniform
    [0, 70000] (raftd's Update takes any Cmd []byte, /root/reference/raft/state_machine.go:126-145)."""
    out = []
    for g in range(G):
        if rng.random() < p_none:
            continue
        n = int(rng.integers(1, nmax + 1))
        pool = list(BIG_LENS) + [0, 1, P, int(rng.integers(0, 70001))]
        lens = [int(x) for x in rng.choice(pool, n)]
        cmds = [rng.integers(0, 256, ln, dtype=np.uint8).tobytes() for ln in lens]
        out.append((base + g, int(rng.integers(0, R)), cmds))
    return out


def cross_check_caller(seed, G, R, T, batches=None, **cfg):
    kw = dict(groups=G, replicas=R, payload_bytes=64, max_entries_per_msg=8, log_capacity=64,
              snapshot_entries=20, compaction_overhead=5, drop_ppm=100000, seed=seed)
    kw.update(cfg)
    a, b = make("c", **kw), make("py", **kw)
    a.bootstrap()
    b.bootstrap()
    rng = np.random.default_rng(seed)
    P = kw["payload_bytes"]
    for t in range(T):
        bt = (batches(rng, G, R, P) if batches else
              random_batches(rng, G, R, kw["max_entries_per_msg"], P, maxc=kw.get("max_cmd_bytes")))
        assert a.propose(bt) == 0 and b.propose(bt) == 0
        _, _, camp, iso = random_inputs(rng, G, R, kw["max_entries_per_msg"])
        a.tick(None, None, camp, iso)
        b.tick(None, None, camp, iso)
        for rid in range(G * R):
            va = a.replica(rid)
            assert va == b.replica(rid), (seed, t, rid)
            for d in range(R):
                assert a.msgs(rid, d) == b.msgs(rid, d), (seed, t, rid, d)
            for i in range(va["marker"] + 1, va["last"] + 1):
                ea = a.entry(rid, i, with_payload=True)
                eb = b.entry(rid, i)
                eb["payload"] = b.reps[rid].log[i - b.reps[rid].marker - 1].data
                assert ea == eb, (seed, t, rid, i)
    return a


@pytest.mark.parametrize("seed", range(6))
def test_caller_proposals_c_matches_python(seed):
    """Variable-length caller Cmds (0, 1, 17, max and random bytes), forwarded by followers to
    their leader with the entries riding in the Propose message: both restatements agree on every
    state, message and entry (payload bytes and CRC over exactly len bytes)."""
    a = cross_check_caller(200 + seed, G=3, R=[1, 2, 3, 5, 3, 4][seed], T=80,
                           payload_bytes=[16, 64, 256, 64, 1024, 32][seed])
    lens = set()
    for rid in range(a.nrep):
        v = a.replica(rid)
        for i in range(v["marker"] + 1, v["last"] + 1):
            e = a.entry(rid, i, with_payload=True)
            lens.add(e["len"])
            if e["len"]:
                import zlib
                assert e["crc"] == zlib.crc32(e["payload"])
    assert 0 in lens and 1 in lens and len(lens) > 3


@pytest.mark.parametrize("seed,R,P,maxc,pages", [(0, 3, 64, 1000, 0), (1, 5, 16, 300, 0), (2, 3, 256, 8191, 0),
                                                  (3, 3, 64, 2000, 16), (4, 1, 1024, 4096, 0)])
def test_long_cmds_c_matches_python(seed, R, P, maxc, pages):
    """Cmds longer than payload_bytes (P - 1, P + 1, max_cmd_bytes, random up to it) in the paged
    payload stream; pages = 16: a short stream, so appends hit the stream capacity rule (DESIGN.md
    §1.7) and both restatements must refuse the same ones."""
    a = cross_check_caller(500 + seed, G=3, R=R, T=60, payload_bytes=P, max_cmd_bytes=maxc, stream_pages=pages)
    lens = set()
    for rid in range(a.nrep):
        v = a.replica(rid)
        for i in range(v["marker"] + 1, v["last"] + 1):
            e = a.entry(rid, i, with_payload=True)
            lens.add(e["len"] if e["type"] == 0 else 0)
            if e["len"] and e["type"] == 0:
                import zlib
                assert e["crc"] == zlib.crc32(e["payload"])
    assert max(lens) > P, lens


@pytest.mark.parametrize("seed,R,P", [(0, 3, 64), (1, 5, 256), (2, 2, 16)])
def test_megabyte_cmds_c_matches_python(seed, R, P):
    """Cmds of 8,191, 8,192, 65,536 and 1 MiB bytes (max_cmd_bytes 1 MiB, far past r03's 8,191-B
    ceiling): stored, forwarded, replicated and CRC'd over exactly their length, identically in both
    restatements, with zlib's CRC-32 of every stored Cmd."""
    import zlib
    a = cross_check_caller(700 + seed, G=3, R=R, T=40, batches=big_batches, payload_bytes=P,
                           max_cmd_bytes=1 << 20)
    lens = set()
    for rid in range(a.nrep):
        v = a.replica(rid)
        for i in range(v["marker"] + 1, v["last"] + 1):
            e = a.entry(rid, i, with_payload=True)
            if e["type"] == 0:
                lens.add(e["len"])
                assert len(e["payload"]) == e["len"] and e["crc"] == (zlib.crc32(e["payload"]) if e["len"] else 0)
    assert {8191, 8192, 65536, 1 << 20} & lens, lens
    assert max(lens) == 1 << 20, lens


def test_cmd_length_limits():
    """max_cmd_bytes up to 16 MiB is accepted, beyond it refused (rg_create's rule); a Cmd longer than
    max_cmd_bytes is refused by or_propose."""
    base = dict(groups=1, replicas=3, payload_bytes=64, max_entries_per_msg=4, log_capacity=64)
    make("c", max_cmd_bytes=1 << 24, **base)
    with pytest.raises(Exception):
        make("c", max_cmd_bytes=(1 << 24) + 1, **base)
    o = make("c", max_cmd_bytes=1000, **base)
    o.bootstrap()
    assert o.propose([(0, 0, [bytes(1001)])]) == -1
    assert o.propose([(0, 0, [bytes(1000)])]) == 0


def lagging_apply(rng, e, nrep, p_notify=0.4):
    """Notify-applied inputs for one tick: each replica, with probability p_notify, reports an
    applied index drawn from [applied, processed] (a state machine that lags, then catches up)."""
    out = []
    for rid in range(nrep):
        v = e.replica(rid)
        if rng.random() < p_notify and v["processed"] >= v["applied"]:
            out.append((rid, int(rng.integers(v["applied"], v["processed"] + 1))))
    return out


@pytest.mark.parametrize("seed", range(4))
def test_apply_feedback_c_matches_python(seed):
    """apply_feedback = 1: `applied` moves only by notify_applied (NotifyRaftLastApplied), so a lagging
    state machine delays campaigns (hasConfigChangeToApply) and snapshots; both restatements agree."""
    kw = dict(groups=3, replicas=[3, 5, 3, 2][seed], payload_bytes=16, max_entries_per_msg=8, log_capacity=64,
              snapshot_entries=20, compaction_overhead=5, drop_ppm=100000, seed=300 + seed, apply_feedback=1)
    a, b = make("c", **kw), make("py", **kw)
    a.bootstrap()
    b.bootstrap()
    rng = np.random.default_rng(seed)
    G, R = kw["groups"], kw["replicas"]
    lagged = 0
    for t in range(120):
        for rid, idx in lagging_apply(rng, a, G * R):
            assert a.notify_applied(rid, idx) == 0 and b.notify_applied(rid, idx) == 0
        assert a.notify_applied(0, a.replica(0)["processed"] + 1) == -1
        ins = random_inputs(rng, G, R, 8)
        a.tick(*ins)
        b.tick(*ins)
        for rid in range(G * R):
            va = a.replica(rid)
            assert va == b.replica(rid), (seed, t, rid)
            for d in range(R):
                assert a.msgs(rid, d) == b.msgs(rid, d), (seed, t, rid, d)
            lagged += va["applied"] < va["committed"]
    assert lagged > 0


def random_reads(rng, G, R, t, p=0.15):
    """ReadIndex requests for one tick: each replica with probability p, a unique non-zero ctx."""
    return [(g, s, (t << 20) | (g * R + s) + 1) for g in range(G) for s in range(R) if rng.random() < p]


@pytest.mark.parametrize("seed", range(5))
def test_read_index_c_matches_python(seed):
    """ReadIndex (Raft thesis §6.4, dragonboat's readIndex): a leader confirms its commit index with a
    heartbeat round carrying the request context, followers forward their requests and get a
    ReadIndexResp; both restatements agree on every message, state and ready read."""
    G, R = 3, [3, 5, 1, 2, 3][seed]
    kw = dict(groups=G, replicas=R, payload_bytes=16, max_entries_per_msg=8, log_capacity=64, snapshot_entries=20,
              compaction_overhead=5, drop_ppm=[100000, 50000, 0, 100000, 0][seed], seed=400 + seed)
    a, b = make("c", **kw), make("py", **kw)
    a.bootstrap()
    b.bootstrap()
    rng = np.random.default_rng(seed)
    ready = 0
    for t in range(120):
        reqs = random_reads(rng, G, R, t)
        assert a.read_index(reqs) == 0 and b.read_index(reqs) == 0
        ins = random_inputs(rng, G, R, 8)
        a.tick(*ins)
        b.tick(*ins)
        for rid in range(G * R):
            assert a.replica(rid) == b.replica(rid), (seed, t, rid)
            for d in range(R):
                assert a.msgs(rid, d) == b.msgs(rid, d), (seed, t, rid, d)
            ra = a.read_ready(rid)
            assert ra == b.read_ready(rid), (seed, t, rid)
            ready += len(ra)
            assert all(ix <= a.replica(rid)["committed"] for _, ix in ra) or a.replica(rid)["role"] != 2
    assert ready > 0


def random_ccs(rng, G, R, p=0.05):
    """Membership changes for one tick: per group, with probability p, add or remove a random slot,
    proposed at a random slot. Removing the last members is a legal input (the group then stalls)."""
    return [(g, int(rng.integers(0, R)), int(rng.choice([1, 2])), int(rng.integers(0, R)))
            for g in range(G) if rng.random() < p]


@pytest.mark.parametrize("seed", range(8))
def test_membership_c_matches_python(seed):
    """ConfigChange proposals (add / remove a slot) under loss, elections and snapshots, from full
    and partial initial memberships: both restatements agree on every view (members, snapshot
    members, pending change), message and entry."""
    G, R = 3, [3, 5, 4, 2, 3, 5, 7, 3][seed]
    kw = dict(groups=G, replicas=R, payload_bytes=16, max_entries_per_msg=8, log_capacity=64, snapshot_entries=20,
              compaction_overhead=5, drop_ppm=[100000, 50000, 0, 100000, 0, 150000, 0, 50000][seed], seed=500 + seed,
              initial_members=[0, 0b01111, 0b0111, 0, 0b011, 0, 0b1011011, 0][seed])
    a, b = make("c", **kw), make("py", **kw)
    a.bootstrap()
    b.bootstrap()
    rng = np.random.default_rng(seed)
    changed = dropped = 0
    for t in range(160):
        for c in random_ccs(rng, G, R):
            ra, rb = a.config_change(*c), b.config_change(*c)
            assert ra == rb == 0, (t, c)
        ins = random_inputs(rng, G, R, 8)
        a.tick(*ins)
        b.tick(*ins)
        for rid in range(G * R):
            va = a.replica(rid)
            assert va == b.replica(rid), (seed, t, rid)
            for d in range(R):
                assert a.msgs(rid, d) == b.msgs(rid, d), (seed, t, rid, d)
            for i in range(va["marker"] + 1, va["last"] + 1):
                assert a.entry(rid, i) == b.entry(rid, i), (seed, t, rid, i)
            changed += va["members"] != (kw["initial_members"] or (1 << R) - 1)
    assert changed > 0


@pytest.mark.parametrize("seed,R,js,im", [(0, 4, 0b1000, 0), (1, 5, 0b11000, 0), (2, 3, 0b100, 0b011),
                                          (3, 4, 0b0110, 0)])
def test_join_slots_c_matches_python(seed, R, js, im):
    """join_slots (StartOnDiskReplica join = true, raft_manager.go:134-144): those slots start empty
    at term 0 outside the membership; random ConfigChanges add them (and remove others) under loss
    and elections; both restatements agree on every view, message and entry."""
    G = 3
    kw = dict(groups=G, replicas=R, payload_bytes=16, max_entries_per_msg=8, log_capacity=64, snapshot_entries=20,
              compaction_overhead=5, drop_ppm=50000, seed=900 + seed, initial_members=im, join_slots=js)
    a, b = make("c", **kw), make("py", **kw)
    a.bootstrap()
    b.bootstrap()
    for rid in range(G * R):
        v = a.replica(rid)
        if js >> (rid % R) & 1:
            assert v["term"] == 0 and v["last"] == 0 and v["members"] == 0, v
        else:
            assert v["members"] == (im or (1 << R) - 1) & ~js and v["last"] == R, v
    rng = np.random.default_rng(seed)
    joiners = [k for k in range(R) if js >> k & 1]
    joined = 0
    for t in range(160):
        ccs = random_ccs(rng, G, R, p=0.05)
        if t % 10 == 5:  # every shard is asked (at a random slot) to add one of its joining slots
            ccs = [(g, int(rng.integers(0, R)), 1, int(rng.choice(joiners))) for g in range(G)]
        for c in ccs:
            assert a.config_change(*c) == b.config_change(*c) == 0, (t, c)
        ins = random_inputs(rng, G, R, 8)
        a.tick(*ins)
        b.tick(*ins)
        for rid in range(G * R):
            va = a.replica(rid)
            assert va == b.replica(rid), (seed, t, rid)
            for d in range(R):
                assert a.msgs(rid, d) == b.msgs(rid, d), (seed, t, rid, d)
            for i in range(va["marker"] + 1, va["last"] + 1):
                assert a.entry(rid, i) == b.entry(rid, i), (seed, t, rid, i)
    for rid in range(G * R):
        v = a.replica(rid)
        joined += (js >> (rid % R) & 1) and (v["members"] >> (rid % R) & 1) and v["last"] > 0
    assert joined > 0


def test_join_scenario():
    """A 2-member shard adds a joining third slot: the joiner stays silent at term 0 until the
    leader's Replicate (or snapshot) reaches it, then holds the leader's log and membership and
    counts toward quorum."""
    from oracle.pyoracle import CC_ADD
    o = make("c", groups=1, replicas=3, payload_bytes=16, max_entries_per_msg=8, log_capacity=256,
             snapshot_entries=0, join_slots=0b100)
    o.bootstrap()
    o.tick()
    o.tick(campaign=np.array([1, 0, 0], np.uint8))
    for _ in range(3):
        o.tick()
    assert o.replica(0)["role"] == 2 and o.replica(0)["members"] == 0b011
    assert o.replica(2)["term"] == 0 and o.replica(2)["last"] == 0
    for _ in range(30):  # not a member: nobody sends it anything, and it never campaigns
        o.tick()
    assert o.replica(2)["term"] == 0 and o.replica(2)["role"] == 0
    assert o.config_change(0, 0, CC_ADD, 2) == 0
    for _ in range(12):  # commit, apply, then a probe round (reject, back to index 1) before the log flows
        o.tick()
    v = [o.replica(r) for r in range(3)]
    assert all(x["members"] == 0b111 for x in v), [x["members"] for x in v]
    assert v[2]["last"] == v[0]["last"] and v[2]["term"] == v[0]["term"]
    iso = np.array([0, 1, 0], np.uint8)  # slot 1 cut off: {0, 2} is a quorum of three
    c0 = v[0]["committed"]
    pt, pc = np.zeros(1, np.uint8), np.ones(1, np.uint32)
    for _ in range(4):
        o.tick(pt, pc, isolate=iso)
    assert o.replica(0)["committed"] >= c0 + 2


def read_heartbeat_drop(o):
    """the leader's read heartbeat is lost (both followers cut off for the tick it is
    sent); the next regular heartbeat carries the pending ctx (dragonboat broadcastHeartbeatMessage
    attaches readIndex.peepCtx), so the read still becomes ready. Returns the ready (ctx, index)."""
    o.bootstrap()
    o.tick()
    o.tick(campaign=np.array([1, 0, 0], np.uint8))
    for _ in range(5):
        o.tick()
    assert o.replica(0)["role"] == 2
    assert o.read_index([(0, 0, 77)]) in (0, None)
    o.tick(isolate=np.array([0, 1, 1], np.uint8))
    assert o.read_ready(0) == []
    hint = None
    for _ in range(6):
        o.tick()
        hb = [m for m in o.msgs(0, 1) if m["type"] == 17]
        if hb and hint is None:
            hint = hb[0]["hint"]
        r = o.read_ready(0)
        if r:
            assert hint == 77  # the regular heartbeat carried the ctx
            return r
    raise AssertionError("the read never became ready")


@pytest.mark.parametrize("kind", ["c", "py"])
def test_read_index_survives_dropped_heartbeat(kind):
    o = make(kind, groups=1, replicas=3, payload_bytes=16, max_entries_per_msg=8, log_capacity=256,
             snapshot_entries=0, heartbeat_rtt=2, election_rtt=20)
    assert [c for c, _ in read_heartbeat_drop(o)] == [77]


def read_queue(o):
    """dragonboat's readIndex queue: five reads reach the leader on consecutive ticks while both
    followers are cut off, so no confirmation round completes. The first four queue up (RG_READ_QUEUE),
    the fifth is dropped and counted. Once the followers are back, the next regular heartbeat carries
    the newest pending ctx (readIndex.peepCtx); its confirmation releases that read and every read
    queued before it, in arrival order, all at its index. Returns (ready reads, drops during the cut)."""
    o.bootstrap()
    o.tick()
    o.tick(campaign=np.array([1, 0, 0], np.uint8))
    for _ in range(5):
        o.tick()
    assert o.replica(0)["role"] == 2
    d0 = o.replica(0)["drops"]
    for k in range(5):
        assert o.read_index([(0, 0, 100 + k)]) in (0, None)
        o.tick(isolate=np.array([0, 1, 1], np.uint8))
        assert o.read_ready(0) == []
    drops = o.replica(0)["drops"] - d0
    for _ in range(6):
        o.tick()
        r = o.read_ready(0)
        if r:
            return r, drops
    raise AssertionError("the queued reads never became ready")


@pytest.mark.parametrize("kind", ["c", "py", "ctl"])
def test_read_index_queue(kind):
    o = make(kind, groups=1, replicas=3, payload_bytes=16, max_entries_per_msg=8, log_capacity=256,
             snapshot_entries=0, heartbeat_rtt=2, election_rtt=20)
    r, drops = read_queue(o)
    assert [c for c, _ in r] == [100, 101, 102, 103] and len({ix for _, ix in r}) == 1
    assert drops >= 1  # the fifth request (messages to the cut-off followers may count too)


def test_membership_scenario():
    """Remove a follower, then the leader, then add both back (3 slots, one group): quorum follows
    the membership, a removed leader steps down, a removed replica never campaigns, an added one
    catches up."""
    from oracle.pyoracle import CC_ADD, CC_REMOVE
    o = make("c", groups=1, replicas=3, payload_bytes=16, max_entries_per_msg=8, log_capacity=256,
             snapshot_entries=0)
    o.bootstrap()
    o.tick()
    o.tick(campaign=np.array([1, 0, 0], np.uint8))
    for _ in range(3):
        o.tick()
    assert o.replica(0)["role"] == 2
    pt, pc = np.zeros(1, np.uint8), np.ones(1, np.uint32)
    assert o.config_change(0, 0, CC_REMOVE, 2) == 0
    assert o.config_change(0, 0, CC_ADD, 1) == -3  # one change per shard per tick
    for _ in range(4):
        o.tick()
    assert [o.replica(r)["members"] for r in range(3)] == [0b011, 0b011, 0b011]  # slot 2 applied it too
    iso = np.array([0, 0, 1], np.uint8)
    c0 = o.replica(0)["committed"]
    for _ in range(4):  # slot 2 cut off: the 2-member quorum {0, 1} still commits
        o.tick(pt, pc, isolate=iso)
    assert o.replica(0)["committed"] >= c0 + 2
    iso = np.array([0, 1, 0], np.uint8)
    for _ in range(2):  # responses slot 1 sent before the cut still arrive
        o.tick(pt, pc, isolate=iso)
    c0 = o.replica(0)["committed"]
    for _ in range(4):  # slot 1 cut off: no quorum of {0, 1}, though slot 2 is reachable
        o.tick(pt, pc, isolate=iso)
    assert o.replica(0)["committed"] == c0
    for _ in range(3):
        o.tick()
    assert o.config_change(0, 1, CC_REMOVE, 0) == 0  # proposed at a follower: forwarded
    for _ in range(5):
        o.tick()
    v = [o.replica(r) for r in range(3)]
    assert v[0]["members"] == 0b010 and v[0]["role"] == 0  # the removed leader stepped down
    for _ in range(40):
        o.tick()
    v = [o.replica(r) for r in range(3)]
    assert v[1]["role"] == 2 and v[0]["role"] != 2 and v[2]["role"] != 2  # sole member leads itself
    c1 = v[1]["committed"]
    o.tick(np.array([1], np.uint8), np.ones(1, np.uint32))
    assert o.replica(1)["committed"] == c1 + 1  # single-node quorum commits on append
    assert o.config_change(0, 1, CC_ADD, 2) == 0
    for _ in range(6):
        o.tick()
    assert o.replica(1)["members"] == 0b110
    o.tick(np.array([1], np.uint8), np.full(1, 4, np.uint32))
    for _ in range(4):
        o.tick()
    assert o.replica(2)["last"] == o.replica(1)["last"] and o.replica(2)["committed"] == o.replica(1)["committed"]


def test_config_change_validation():
    for kind in ("c", "py"):
        o = make(kind, groups=2, replicas=3, payload_bytes=16)
        o.bootstrap()
        assert o.config_change(2, 0, 1, 0) == -1   # no such group
        assert o.config_change(0, 3, 1, 0) == -1   # no such slot
        assert o.config_change(0, 0, 1, 3) == -1   # no such target
        assert o.config_change(0, 0, 3, 0) == -1   # no such op
        assert o.config_change(0, 0, 2, 1) == 0
        assert o.config_change(0, 1, 1, 1) == -3   # one per shard per tick
        assert o.config_change(1, 1, 1, 1) == 0


def test_propose_validation():
    o = pyoracle.Oracle(groups=2, replicas=3, payload_bytes=16, max_entries_per_msg=4)
    py = make("py", groups=2, replicas=3, payload_bytes=16, max_entries_per_msg=4)
    for e in (o, py):
        e.bootstrap()
        assert e.propose([(0, 1, [b"a"] * 3)]) == 0
        assert e.propose([(0, 1, [b"b"] * 2)]) == -3  # 5 > E in one tick
        assert e.propose([(0, 2, [b"c"])]) == -3      # second slot of one group
        assert e.propose([(1, 0, [b"x" * 17])]) == -1  # Cmd longer than payload_bytes
        assert e.propose([(2, 0, [b"x"])]) == -1       # no such group
        assert e.propose([(1, 0, [])]) == -1           # empty batch
        assert e.propose([(1, 0, [b"ok"]), (1, 0, [b"x" * 99])]) == -1  # all or nothing
        assert e.propose([(0, 1, [b"d"])]) == 0        # 4 = E
    with pytest.raises(ValueError):
        o.tick(np.zeros(2, np.uint8), np.ones(2, np.uint32))  # one proposal source per tick


@pytest.mark.parametrize("seed", range(10))
def test_c_oracle_matches_python_restatement(seed):
    cross_check(seed, G=3, R=[1, 2, 3, 4, 5][seed % 5], T=100)


@pytest.mark.parametrize("seed", range(3))
def test_c_oracle_matches_python_no_loss_r7(seed):
    cross_check(100 + seed, G=2, R=7, T=60, drop_ppm=0, max_msgs_per_pair=4)


@pytest.mark.parametrize("name", ["trace_r3_chaos.json", "trace_r5_chaos.json"])
def test_regression_traces(name):
    fx = K.load(name)
    o = pyoracle.Oracle(**fx["config"])
    o.bootstrap()
    rng = np.random.default_rng(fx["input_seed"])
    G, R = o.G, o.R
    for t in range(fx["ticks"]):
        o.tick(*random_inputs(rng, G, R, fx["config"]["max_entries_per_msg"]))
        h = hashlib.sha256()
        for rid in range(G * R):
            h.update(json.dumps(o.replica(rid), sort_keys=True).encode())
            for d in range(R):
                h.update(json.dumps(o.msgs(rid, d), sort_keys=True).encode())
        assert h.hexdigest()[:16] == fx["digests"][t], t
    assert [o.replica(r) for r in range(G * R)] == fx["final"]


def test_steady_state_throughput_shape():
    """C2-shaped steady state: every group elects slot 0 and commits every proposal batch."""
    G, R, E = 8, 3, 16
    o = pyoracle.Oracle(groups=G, replicas=R, payload_bytes=64, max_entries_per_msg=E)
    o.bootstrap()
    o.tick()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    o.tick(campaign=camp)
    for _ in range(40):
        o.tick(np.zeros(G, np.uint8), np.full(G, E, np.uint32), threads=4)
    for g in range(G):
        v = o.replica(g * R)
        assert v["role"] == 2 and v["term"] == 2
        assert v["committed"] >= v["last"] - 2 * E
        for s in range(1, R):
            f = o.replica(g * R + s)
            assert f["role"] == 0 and f["leader"] == 1 and f["err"] == 0


def _digest_py(o, R):
    """or_digest restated from the oracle's public views."""
    M = (1 << 64) - 1

    def mix(z):
        z ^= z >> 33
        z = (z * 0xFF51AFD7ED558CCD) & M
        z ^= z >> 33
        z = (z * 0xC4CEB9FE1A85EC53) & M
        return z ^ (z >> 33)

    a = b = 0
    base = o.cfg["group_base"]
    for rid in range(o.nrep):
        v = o.replica(rid)
        gid = (base + rid // R) * R + rid % R
        h = mix((gid + 0x9E3779B97F4A7C15) & M)
        for f in ("term", "vote", "leader", "committed", "applied", "last", "marker", "marker_term", "snap_index",
                  "snap_term", "cap_base", "processed", "role", "election_tick", "heartbeat_tick", "rand_timeout",
                  "rng_ctr", "granted", "responded", "active", "err", "drops", "members", "snap_members",
                  "cc_pending"):
            h = mix(h ^ v[f])
        for j in range(R):
            for f in ("match", "next", "rsnap", "rstate"):
                h = mix(h ^ v[f][j])
        a = (a + h) & M
        h2 = mix(gid ^ 0x5851F42D4C957F2D)
        for i in range(v["marker"] + 1, v["last"] + 1):
            en = o.entry(rid, i)
            h2 = mix(h2 ^ en["term"])
            h2 = mix(h2 ^ (en["type"] | (en["len"] << 8) | (en["crc"] << 32)))
        b = (b + h2) & M
    return a, b


def test_digest_definition_and_windows():
    """or_digest equals its restatement from the public views, and the digests of group windows add
    up to the digest of their union (what lets a rank or a window be checked on its own)."""
    import numpy as np
    G, R = 8, 3
    cfg = dict(replicas=R, log_capacity=64, payload_bytes=32, max_entries_per_msg=8, snapshot_entries=20,
               compaction_overhead=3, drop_ppm=30000, seed=0xD16)
    whole = make("c", groups=G, **cfg)
    halves = [make("c", groups=G // 2, group_base=b, **cfg) for b in (0, G // 2)]
    for o in [whole] + halves:
        o.bootstrap()
    rng = np.random.default_rng(2)
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    for t in range(40):
        pt = rng.integers(0, R, G).astype(np.uint8)
        pc = rng.integers(1, 9, G).astype(np.uint32)
        ins = dict(campaign=camp) if t == 1 else dict(prop_target=pt, prop_count=pc) if t > 4 else {}
        whole.tick(**ins)
        for k, o in enumerate(halves):
            sl = slice(k * G // 2, (k + 1) * G // 2)
            o.tick(**{n: (v[k * G // 2 * R:(k + 1) * G // 2 * R] if n == "campaign" else v[sl]) for n, v in ins.items()})
    d = whole.digest()
    assert d == _digest_py(whole, R)
    s = [sum(x) & ((1 << 64) - 1) for x in zip(*(o.digest() for o in halves))]
    assert tuple(s) == d
    assert whole.replica(0)["snap_index"] > 0  # compaction happened: the log chains start above a marker


@pytest.mark.parametrize("seed", range(4))
def test_compact_c_matches_python(seed):
    """rg_compact's restatement (or_compact / Sim.compact): between ticks random shards compact to a
    random index — capped at each replica's snapshot index, ignored at or below its marker — and both
    restatements agree on the count, every replica, message and entry (lagging followers then get
    InstallSnapshot; the stream below is released by the next step)."""
    G, R = 4, [3, 5, 3, 2][seed]
    kw = dict(groups=G, replicas=R, payload_bytes=16, max_entries_per_msg=8, log_capacity=64, snapshot_entries=12,
              compaction_overhead=5, drop_ppm=100000, seed=700 + seed)
    a, b = make("c", **kw), make("py", **kw)
    a.bootstrap()
    b.bootstrap()
    rng = np.random.default_rng(seed)
    moved = 0
    for t in range(120):
        for g in range(G):
            if rng.random() < 0.3:
                idx = int(rng.integers(0, a.replica(g * R)["committed"] + 6))
                na, nb = a.compact(g, idx), b.compact(g, idx)
                assert na == nb, (seed, t, g, idx)
                moved += na
        assert a.compact(G, 5) == -1 and b.compact(G, 5) == -1
        ins = random_inputs(rng, G, R, 8)
        a.tick(*ins)
        b.tick(*ins)
        for rid in range(G * R):
            va = a.replica(rid)
            assert va == b.replica(rid), (seed, t, rid)
            for d in range(R):
                assert a.msgs(rid, d) == b.msgs(rid, d), (seed, t, rid, d)
            for i in range(va["marker"] + 1, va["last"] + 1):
                assert a.entry(rid, i) == b.entry(rid, i), (seed, t, rid, i)
    assert moved > 10
