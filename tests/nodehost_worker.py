"""Worker of test_nodehost's multi-process test: N processes (one rank = one raftd node each, gloo)
run one raftd_amd.nodehost.NodeHost per node over their DistEngine share of an N-rank cluster on the
same GPU (replicas = N: one replica of every shard per node).

Every node starts its replica of every shard itself — the first N-1 nodes as initial members, the
last with join = true (raft/raft_manager.go:134-144); after the elections node 0 recruits the last
node into every shard, later node 1 removes node 0 from the even shards. Each tick every rank
all-gathers its staged membership inputs and its replicas' views; rank 0 replays the starts and the
inputs on the C oracle of the whole shard set and compares every replica, every tick.
usage: python nodehost_worker.py N"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]

import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

G_LOCAL, TICKS = 4, 150
NODES = [(11, "n0:63001"), (22, "n1:63001"), (33, "n2:63001"), (44, "n3:63001")]


def cfg(n):
    return dict(replicas=n, log_capacity=128, payload_bytes=16, max_entries_per_msg=8, snapshot_entries=40,
                compaction_overhead=4, drop_ppm=20000, seed=0x90DE)


def start(nh, G, n):
    initial = dict(NODES[:n - 1])
    for g in range(G):
        join = nh.replica_id not in initial
        nh.StartOnDiskReplica(None if join else initial, join, None, {"ShardID": g})


def worker(rank, n):
    dist.init_process_group("gloo", rank=rank, world_size=n)
    from raftd_amd.cluster import DistEngine
    from raftd_amd.nodehost import NodeHost
    de = DistEngine(groups=G_LOCAL, device=0, **cfg(n))
    de.bootstrap()
    G, R = G_LOCAL * n, n
    nh = NodeHost(de, R, NODES[:n])
    start(nh, G, n)
    last_id, first_id = NODES[n - 1][0], NODES[0][0]
    reqs = []
    log = []
    for t in range(TICKS):
        if t == 35 and rank == 0:
            reqs += [nh.RequestAddReplica(g, last_id, NODES[n - 1][1], deadline_ticks=80) for g in range(G)]
        if t == 90 and rank == 1:
            reqs += [nh.RequestDeleteReplica(g, first_id, deadline_ticks=50) for g in range(0, G, 2)]
        nh.step()
        mine = {g * R + s: nh.h.replica_of(g, s) for g in range(G) for s in range(R) if nh.h.hosts(g, s)}
        allx = [None] * n
        dist.all_gather_object(allx, (nh.staged, mine))
        log.append(allx)
    assert all(r.done for r in reqs), [(r.shard, r.op, r.error) for r in reqs if not r.done]
    for g in range(G):
        if rank == 0 and g % 2 == 0:
            continue  # node 0 left the even shards: no leader talks to its replica any more
        lid, term, valid = nh.GetLeaderID(g)
        want = {i: a for i, a in NODES[:n] if not (g % 2 == 0 and i == first_id)}
        assert valid and lid in want, (rank, g, lid, valid)
        m = nh.SyncGetShardMembership(g).nodes
        assert m == want, (rank, g, m, want)
    if rank == 0:
        from oracle.pyoracle import Oracle
        from raftd_amd.cluster import RankView
        ora = Oracle(groups=G, **cfg(n))
        ora.bootstrap()
        for k in range(n):  # every node's start, replayed on the oracle
            start(NodeHost(RankView(ora, k, n, R), R, NODES[:n]), G, n)
        for t in range(TICKS):
            for staged, _ in log[t]:
                for g, s, op, target in staged:
                    assert ora.config_change(g, s, op, target) == 0
            ora.tick()
            for _, mine in log[t]:
                for rid, v in mine.items():
                    ov = ora.replica(rid)
                    assert v == ov, (t, rid, {k: (v[k], ov[k]) for k in ov if v[k] != ov[k]})
        print(f"nodehost parity ok: {n} nodes, {G} shards, {TICKS} ticks", flush=True)
    de.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    n = int(sys.argv[1])
    mp.spawn(worker, args=(n,), nprocs=n, join=True)
