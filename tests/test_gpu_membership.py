"""Membership changes through the C-ABI (rg_config_change) against the oracle (or_config_change).

raftd's RaftManager.RecruitReplica / RemoveReplica call NodeHost.SyncRequestAddReplica /
SyncRequestDeleteReplica (/root/reference/raft/raft_manager.go:165-185), and StartOnDiskReplica
takes the initial members (:114-144). Here a ConfigChange entry is proposed at a replica, forwarded
by followers (across ranks too), replicated, and applied when it is handed to each replica's state
machine; quorum, elections, replication, ReadIndex and snapshots then follow the new membership
(DESIGN.md §1.8). Every view (members, snapshot members, pending change), message and entry must
equal the oracle's. Parity with dragonboat itself is unpinned.
"""
import numpy as np
import pytest

from engines import make
from test_gpu_parity import CHAOS, compare, random_inputs
from test_gpu_propose import check_applied
from test_oracle import random_batches, random_ccs

pytestmark = pytest.mark.gpu


def run_members(cfg, ticks, seed, make_gpu=None, p_cc=0.06, caller=False):
    gpu = make_gpu() if make_gpu else make("gpu", **cfg)
    ora = make("c", **cfg)
    gpu.bootstrap()
    ora.bootstrap()
    rng = np.random.default_rng(seed)
    G, R = ora.G, ora.R
    im = cfg.get("initial_members", 0) or (1 << R) - 1
    changed = 0
    for t in range(ticks):
        for c in random_ccs(rng, G, R, p_cc):
            assert ora.config_change(*c) == 0
            gpu.config_change(*c)
        if caller:
            b = random_batches(rng, G, R, cfg["max_entries_per_msg"], cfg["payload_bytes"])
            gpu.propose(b)
            assert ora.propose(b) == 0
            _, _, camp, iso = random_inputs(rng, G, R, cfg["max_entries_per_msg"])
            ins = (None, None, camp, iso)
        else:
            ins = random_inputs(rng, G, R, cfg["max_entries_per_msg"])
        gpu.tick(*ins)
        ora.tick(*ins)
        compare(gpu, ora, t)
        if caller and hasattr(gpu, "apply_committed"):
            check_applied(gpu, ora)  # ConfigChange entries never reach Update
        changed += sum(ora.replica(r)["members"] != im for r in range(G * R))
    assert changed > 0
    return gpu, ora


@pytest.mark.parametrize("R,im,drop", [(3, 0, 150000), (5, 0b01011, 150000), (2, 0b01, 150000), (8, 0, 50000),
                                       (4, 0b0111, 150000)])
def test_membership_chaos(R, im, drop):
    """(At R = 8 with 15 % loss leadership rarely lasts long enough to commit a change: 5 % there.)"""
    cfg = dict(CHAOS, groups=4, replicas=R, payload_bytes=16, max_entries_per_msg=8, seed=800 + R,
               initial_members=im, drop_ppm=drop)
    run_members(cfg, ticks=150, seed=R, p_cc=0.08 if R == 8 else 0.06)


def test_membership_with_caller_cmds():
    cfg = dict(CHAOS, groups=4, replicas=3, payload_bytes=64, max_entries_per_msg=8, seed=81)
    run_members(cfg, ticks=120, seed=9, caller=True)


@pytest.mark.parametrize("R,js,im", [(4, 0b1000, 0), (5, 0b11000, 0), (3, 0b100, 0b011)])
def test_join_slots(R, js, im):
    """join_slots (StartOnDiskReplica join = true): empty joiners at term 0 outside the membership,
    added by ConfigChanges every 10 ticks, catch up through probing (or a snapshot) bit-exact with
    the oracle."""
    cfg = dict(CHAOS, groups=4, replicas=R, payload_bytes=16, max_entries_per_msg=8, seed=950 + R,
               initial_members=im, join_slots=js, drop_ppm=50000)
    gpu, ora = make("gpu", **cfg), make("c", **cfg)
    gpu.bootstrap()
    ora.bootstrap()
    compare(gpu, ora, -1)
    rng = np.random.default_rng(R)
    G = 4
    joiners = [k for k in range(R) if js >> k & 1]
    for t in range(150):
        ccs = random_ccs(rng, G, R, 0.04)
        if t % 10 == 5:
            ccs = [(g, int(rng.integers(0, R)), 1, int(rng.choice(joiners))) for g in range(G)]
        for c in ccs:
            assert ora.config_change(*c) == 0
            gpu.config_change(*c)
        ins = random_inputs(rng, G, R, cfg["max_entries_per_msg"])
        gpu.tick(*ins)
        ora.tick(*ins)
        compare(gpu, ora, t)
    joined = sum(1 for r in range(G * R) if js >> (r % R) & 1 and ora.replica(r)["members"] >> (r % R) & 1
                 and ora.replica(r)["last"] > 0)
    assert joined > 0


@pytest.mark.parametrize("ranks,R", [(2, 3), (3, 5)])
def test_membership_cluster(ranks, R):
    """Changes proposed at followers on other ranks are forwarded over the wire; InstallSnapshot
    carries the snapshot's membership across ranks."""
    from raftd_amd.cluster import LoopbackCluster
    cfg = dict(CHAOS, groups=2 * ranks, replicas=R, payload_bytes=16, max_entries_per_msg=8, seed=30 + ranks)
    run_members(cfg, ticks=120, seed=ranks * 3 + R, make_gpu=lambda: LoopbackCluster(ranks=ranks, **cfg))


def test_membership_survives_wal_restart(tmp_path):
    """The persisted state records carry the membership; a node restarted from its WAL comes back
    with it, and re-applying the ConfigChange entries above the app's index changes nothing."""
    from raftd_amd.wal import WAL, replay, restore
    cfg = dict(CHAOS, groups=4, replicas=3, payload_bytes=16, max_entries_per_msg=8, seed=83, drop_ppm=0)
    full = dict(cfg, election_rtt=10, heartbeat_rtt=1)
    gpu = make("gpu", **cfg)
    gpu.bootstrap()
    wal = WAL(str(tmp_path / "node.wal"))
    wal.append(0, *gpu.persist_collect(full=True), cfg["payload_bytes"])
    rng = np.random.default_rng(4)
    G, R = 4, 3
    for t in range(60):
        for c in random_ccs(rng, G, R, 0.08):
            gpu.config_change(*c)
        gpu.tick(*random_inputs(rng, G, R, 8))
        wal.append(t + 1, *gpu.persist_collect(), cfg["payload_bytes"])
    before = [gpu.replica(r)["members"] for r in range(G * R)]
    assert any(m != 0b111 for m in before)
    logs = replay(wal.path, R)
    g2, ora = make("gpu", **cfg), make("c", **cfg)
    g2.bootstrap()
    ora.bootstrap()
    rids = [(r, r) for r in range(G * R)]
    restore(g2, logs, full, rids)
    restore(ora, logs, full, rids)
    assert [g2.replica(r)["members"] for r in range(G * R)] == before
    compare(g2, ora, -1)
    for t in range(20):
        ins = random_inputs(rng, G, R, 8)
        g2.tick(*ins)
        ora.tick(*ins)
        compare(g2, ora, t)


def test_config_change_errors():
    from raftd_amd.engine import CC_ADD, CC_REMOVE, RG_EFULL, RG_EINVAL, RgError
    gpu = make("gpu", groups=2, replicas=3, payload_bytes=16)
    gpu.bootstrap()
    for args in ((2, 0, CC_ADD, 0), (0, 3, CC_ADD, 0), (0, 0, CC_ADD, 3), (0, 0, 3, 0)):
        with pytest.raises(RgError) as ei:
            gpu.config_change(*args)
        assert ei.value.code == RG_EINVAL, args
    gpu.config_change(0, 0, CC_REMOVE, 1)
    with pytest.raises(RgError) as ei:
        gpu.config_change(0, 1, CC_ADD, 1)
    assert ei.value.code == RG_EFULL
    gpu.tick()
    gpu.config_change(0, 1, CC_ADD, 1)  # the staging resets after the tick that carried it
