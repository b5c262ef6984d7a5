"""The deliberate departures from dragonboat's step ("Departures from dragonboat"), one
test per row, on the CPU restatements (the C oracle, and the Python one as a cross-check). Each rule is
a place where the restatement's message set or log can differ from dragonboat's on some trace; each
test builds that trace and shows the rule is reported — counted in the replica's `drops`, flagged in
its `err` word, or visible in the message itself — never silent. This is what makes "bit-exact with
this restatement" checkable: on a recorded dragonboat trace, a non-zero counter names the rule that
made the two diverge. drop_ppm is 0 throughout, so every drop counted here is the rule's."""
import numpy as np
import pytest

from engines import make, view

PROPOSE, READ_INDEX, REPL, HEARTBEAT, RV = 7, 19, 12, 17, 14
TERM_MASK = (1 << 36) - 1
ERR_TERM_LIMIT = 128


def cluster(kind, **kw):
    """One shard of three replicas, slot 0 elected (bootstrap, one tick, campaign, four ticks)."""
    cfg = dict(groups=1, replicas=3, log_capacity=256, payload_bytes=16, max_entries_per_msg=8,
               max_msgs_per_pair=4, drop_ppm=0, snapshot_entries=0, seed=0xD1F)
    cfg.update(kw)
    e = make(kind, **cfg)
    e.bootstrap()
    e.tick()
    e.tick(campaign=np.array([1, 0, 0], np.uint8))
    for _ in range(4):
        e.tick()
    assert e.replica(0)["role"] == 2 and e.replica(1)["leader"] == 1
    return e


def propose(n):
    return np.array([0], np.uint8), np.array([n], np.uint32)


@pytest.mark.parametrize("kind", ["c", "py"])
def test_replicate_entry_count_limit(kind):
    """a9: a Replicate carries at most max_entries_per_msg entries (dragonboat: a byte budget). A follower
    lagging by more than E entries is caught up by several Replicates; each full one is visible as
    nent == E with the leader's log running past it."""
    E = 4
    e = cluster(kind, max_entries_per_msg=E)
    iso = np.zeros(3, np.uint8)
    iso[2] = 1
    for _ in range(4):  # slot 2 misses 16 entries
        e.tick(*propose(E), isolate=iso)
    split = 0
    for _ in range(20):
        e.tick()
        last = e.replica(0)["last"]
        for m in e.msgs(0, 2):
            if m["type"] == REPL:
                assert m["nent"] <= E
                split += m["nent"] == E and m["log_index"] + m["nent"] < last
    assert split >= 1, "the catch-up never needed a second Replicate"
    assert e.replica(2)["last"] == e.replica(0)["last"]


@pytest.mark.parametrize("kind", ["c", "py"])
def test_k_max_messages_per_pair_drops_are_counted(kind):
    """K_MAX: at most max_msgs_per_pair messages from one replica to another per tick; the excess is dropped
    and counted in the sender's drops (dragonboat's transport queue is deeper). A leader with a batch sends
    each follower a Replicate and a Heartbeat per tick, and another Replicate when an ack moves its commit:
    K = 1 drops at least one of them every tick, K = 4 (the default) none."""
    drops = {}
    for K in (1, 4):
        e = cluster(kind, max_msgs_per_pair=K)
        d0 = e.replica(0)["drops"]
        for _ in range(5):
            e.tick(*propose(2))
        drops[K] = e.replica(0)["drops"] - d0
    assert drops[4] == 0
    assert drops[1] >= 5 * 2  # two followers, at least one message each per tick


@pytest.mark.parametrize("kind", ["c"])
def test_forward_hop_limit_is_counted(kind):
    """A proposal is forwarded at most once (hop 0 -> 1): a follower receiving an already-forwarded Propose
    drops it and counts it (dragonboat forwards to whatever it believes the leader is)."""
    e = cluster(kind)
    d0 = e.replica(2)["drops"]
    e.deliver(1, type=PROPOSE, to=3, term=0, nent=1, src_a=0, src_b=1)
    e.tick(flags=1)  # no timers: only the delivered message
    assert e.replica(2)["drops"] == d0 + 1
    assert not any(m["type"] == PROPOSE for m in e.msgs(2, 0))


@pytest.mark.parametrize("kind", ["c", "py"])
def test_term_limit_is_flagged(kind):
    """Terms are 36-bit (they share the ring word with the Cmd length): a campaign at term 2^36 - 1 is
    refused and flagged RG_ERR_TERM_LIMIT in the replica's err word, the term unchanged."""
    cfg = dict(groups=1, replicas=3, log_capacity=64, payload_bytes=16, max_entries_per_msg=8, drop_ppm=0)
    e = make(kind, **cfg)
    e.bootstrap()
    e.import_replica(1, view(3, term=TERM_MASK, last=1, next=[2] * 3), [TERM_MASK])
    e.tick(campaign=np.array([0, 1, 0], np.uint8))
    r = e.replica(1)
    assert r["err"] & ERR_TERM_LIMIT and r["term"] == TERM_MASK and r["role"] != 1


@pytest.mark.parametrize("kind", ["c", "py"])
def test_read_index_queue_overflow_is_counted(kind):
    """The leader's ReadIndex queue holds RG_READ_QUEUE = 4 pending requests; a fifth is dropped and counted
    (dragonboat's queue is unbounded). The followers are isolated so no request is confirmed: five reads
    count exactly one drop more than four over the same five ticks (the isolation's own losses are equal)."""
    got = {}
    for n in (4, 5):
        e = cluster(kind)
        iso = np.array([0, 1, 1], np.uint8)
        d0 = e.replica(0)["drops"]
        for t in range(5):
            if t < n:
                e.read_index([(0, 0, 1000 + t)])
            e.tick(isolate=iso)
        got[n] = e.replica(0)["drops"] - d0
    assert got[5] == got[4] + 1


@pytest.mark.parametrize("kind", ["c", "py"])
def test_ring_capacity_refusals_are_counted(kind):
    """A replica holds at most log_capacity entries above its last compaction (dragonboat's log is
    unbounded in LogDB): a leader batch that would pass cap_base + L is refused whole and counted."""
    L, E = 16, 8
    e = cluster(kind, log_capacity=L, max_entries_per_msg=E, snapshot_entries=0)
    d0, last0 = e.replica(0)["drops"], e.replica(0)["last"]
    for _ in range(4):
        e.tick(*propose(E))
    r = e.replica(0)
    assert r["last"] <= r["cap_base"] + L
    refused = 4 - (r["last"] - last0) // E
    assert refused >= 1 and r["drops"] - d0 == refused


@pytest.mark.parametrize("kind", ["c", "py"])
def test_inbox_order_is_sender_slot_order(kind):
    """Messages of one tick are handled in ascending sender slot (dragonboat: transport arrival order, and
    its broadcasts walk a Go map). Two candidates of the same term ask a fresh voter in one tick: the lower
    slot's request is handled first and gets the vote, whichever was delivered first."""
    for first, second in ((0, 2), (2, 0)):
        e = make(kind, groups=1, replicas=3, log_capacity=64, payload_bytes=16, max_entries_per_msg=8, drop_ppm=0)
        e.bootstrap()
        e.import_replica(1, view(3, term=1, last=1, next=[2] * 3), [1])
        for src in (first, second):
            e.deliver(src, type=RV, to=2, term=2, log_term=1, log_index=1)
        e.tick(flags=1)
        assert e.replica(1)["vote"] == 1, (first, second)  # slot 0 (id 1) won


def test_departure_table_lists_every_tested_rule():
    """DESIGN.md §5's table names each rule this file tests (and the counter that reports it)."""
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    text = open(os.path.join(root, "DESIGN.md")).read()
    sec = text[text.index("### Departures from dragonboat"):]
    sec = sec[:sec.index("\n## ")]
    for name in ("test_replicate_entry_count_limit", "test_k_max_messages_per_pair_drops_are_counted",
                 "test_forward_hop_limit_is_counted", "test_term_limit_is_flagged",
                 "test_read_index_queue_overflow_is_counted", "test_ring_capacity_refusals_are_counted",
                 "test_inbox_order_is_sender_slot_order"):
        assert name in sec, name
