"""Hosting the step engine on several ranks: placement math, the per-tick message
exchange, and two drivers over the C-ABI's transport plug (rg_wire_plan / rg_wire_pack /
rg_wire_recv in include/raftgpu.h).

Replicas of one Raft group live on different ranks, emulating raftd's separate nodes (each node
runs one dragonboat NodeHost, /root/reference/raft/raft_manager.go:102-109). dragonboat sends a
replica's outbound pb.Messages to its transport after the step; here every message emitted in
tick t to a replica on another rank travels in one batch before tick t+1, one region per rank
pair.

- ``DistEngine``: one rank per process (``torch.distributed``). With the ``nccl`` backend (RCCL on
  ROCm) the regions move GPU to GPU by one ``all_to_all_single`` over xGMI per tick — the only
  collective of the data path; with ``gloo`` they are staged through host memory (tests).
- ``LoopbackCluster``: N ranks as N engines in one process on one GPU, regions moved by device
  copies. Exposes the single-engine interface in GLOBAL replica ids, so parity tests compare a
  sharded cluster with the oracle of the whole shard set.
"""
from __future__ import annotations

from .engine import Engine, default_config


# ---------------------------------------------------------------- placement (raftgpu_internal.h)
def slot_offset(s: int, j: int, n: int) -> int:
    """off_c(s): rank offset of slot s in column j (class c = j mod (n - 1)); 0 for slot 0."""
    if s == 0 or n < 2:
        return 0
    m = n - 1
    return (j % m + s - 1) % m + 1


def rank_of(g: int, s: int, n: int) -> int:
    """Rank hosting slot s of global group g."""
    return (g % n + slot_offset(s, g // n, n)) % n


def local_rid(g: int, s: int, n: int, replicas: int) -> int:
    """Local replica id (column * R + slot) of slot s of global group g on its rank."""
    return (g // n) * replicas + s


def global_group(rank: int, s: int, j: int, n: int) -> int:
    """Global group of local replica (slot s, column j) on `rank` (pl_group)."""
    return n * j + (rank - slot_offset(s, j, n)) % n


def plane_offset(s: int, d: int, j: int, n: int) -> int:
    """Rank offset of the outbox plane s→d in column j (pl_off; 0 = co-located)."""
    return (slot_offset(d, j, n) - slot_offset(s, j, n)) % n


def _torch():
    import torch
    return torch


class _Buf:
    """A growable device byte buffer (torch allocation; the engine only sees the pointer)."""

    def __init__(self, device):
        self.device = device
        self.t = None

    def ensure(self, n: int):
        torch = _torch()
        if self.t is None or self.t.numel() < n:
            cap = max(n, 1 << 20)
            if self.t is not None:
                cap = max(cap, int(self.t.numel() * 1.5))
            self.t = torch.empty(cap, dtype=torch.uint8, device=self.device)
        return self.t

    def ptr(self) -> int:
        return self.t.data_ptr() if self.t is not None else 0

    def cap(self) -> int:
        return self.t.numel() if self.t is not None else 0


def _offsets(sizes):
    out, o = [], 0
    for n in sizes:
        out.append(o)
        o += n
    return out, o


# ---------------------------------------------------------------- one process per rank
def all_to_all_bytes(send, send_sizes, recv, recv_sizes, group=None):
    """Move region r of `send` (sizes send_sizes, concatenated in rank order) to rank r; the
    regions from every rank land concatenated in rank order in `recv`. nccl: device tensors, one
    all_to_all_single (RCCL over xGMI). gloo: staged through host memory."""
    import torch.distributed as dist
    torch = _torch()
    stot, rtot = sum(send_sizes), sum(recv_sizes)
    if dist.get_backend(group) == "nccl":
        dist.all_to_all_single(recv[:rtot], send[:stot], list(recv_sizes), list(send_sizes), group=group)
        return
    hs = send[:stot].cpu() if send.is_cuda else send[:stot]
    hr = torch.empty(rtot, dtype=torch.uint8)
    dist.all_to_all_single(hr, hs, list(recv_sizes), list(send_sizes), group=group)
    recv[:rtot].copy_(hr)


def exchange_sizes(send_sizes, group=None):
    """Each rank's outbound region sizes → the sizes this rank receives from every rank."""
    import torch.distributed as dist
    torch = _torch()
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    st = torch.tensor(send_sizes, dtype=torch.int64, device=dev)
    rt = torch.empty_like(st)
    dist.all_to_all_single(rt, st, group=group)
    return [int(x) for x in rt.tolist()]


class DistEngine:
    """This process's engine of an N-rank cluster (rank = torch.distributed rank). `groups` is
    the number of local columns (the cluster hosts ranks * groups shards). The engine launches
    on torch's current stream, so the exchange orders itself behind the tick that produced it."""

    def __init__(self, groups: int, group=None, **cfg):
        import torch.distributed as dist
        torch = _torch()
        self.pg = group
        self.N, self.rank = dist.get_world_size(group), dist.get_rank(group)
        self.eng = Engine(groups=groups, ranks=self.N, rank=self.rank, **cfg)
        torch.cuda.set_device(self.eng.cfg["device"])
        self.stream = torch.cuda.current_stream()
        if self.stream.cuda_stream == 0:  # the engine needs a real stream shared with torch's copies
            self.stream = torch.cuda.Stream()
            torch.cuda.set_stream(self.stream)
        self.eng.set_stream(self.stream.cuda_stream)
        dev = torch.device("cuda", self.eng.cfg["device"])
        self.send, self.recv = _Buf(dev), _Buf(dev)
        self.wire_bytes = 0  # bytes this rank sent in the last exchange

    def exchange(self):
        """Ship the last tick's cross-rank messages (before every tick)."""
        e = self.eng
        sizes = e.wire_plan()
        _, stot = _offsets(sizes)
        self.send.ensure(stot)
        e.wire_pack(self.send.ptr(), self.send.cap())
        rsizes = exchange_sizes(sizes, self.pg)
        _, rtot = _offsets(rsizes)
        if rtot > self.recv.cap():
            e.sync()  # the previous tick's followers may still read the old receive buffer
        self.recv.ensure(rtot)
        all_to_all_bytes(self.send.t, sizes, self.recv.t, rsizes, self.pg)
        e.wire_recv(self.recv.ptr(), rsizes)
        self.wire_bytes = stot - sizes[self.rank]

    def tick(self, *a, **kw):
        self.exchange()
        self.eng.tick(*a, **kw)

    def tick_device(self, *a, **kw):
        self.exchange()
        self.eng.tick_device(*a, **kw)


# ---------------------------------------------------------------- N ranks in one process
class LoopbackCluster:
    """N engines (ranks) in one process on one GPU, moving regions with device copies. The
    interface is the single Engine's, in GLOBAL ids: replica id g * R + s, `groups` = all
    ranks' shards (a multiple of ranks)."""

    def __init__(self, ranks: int, groups: int, **cfg):
        torch = _torch()
        if groups % ranks:
            raise ValueError("groups must be a multiple of ranks")
        self.N = ranks
        self.cfg = default_config(groups=groups, **cfg)
        self.G, self.R = groups, self.cfg["replicas"]
        self.nrep = self.G * self.R
        lc = dict(self.cfg, groups=groups // ranks)
        self.engines = [Engine(**dict(lc, ranks=ranks, rank=k)) for k in range(ranks)]
        dev = torch.device("cuda", self.cfg["device"])
        self.send = [_Buf(dev) for _ in range(ranks)]
        self.recv = [_Buf(dev) for _ in range(ranks)]
        self.loc = [None] * self.nrep  # global rid → (rank, local rid)
        for k, e in enumerate(self.engines):
            for lr in range(e.nrep):
                g, gr = e.global_id(lr)
                self.loc[gr] = (k, lr)
        self.wire_bytes = 0

    def close(self):
        for e in self.engines:
            e.close()

    def bootstrap(self):
        for e in self.engines:
            e.bootstrap()

    def exchange(self):
        torch = _torch()
        sizes = [e.wire_plan() for e in self.engines]  # sizes[a][b]: rank a → rank b
        for k, e in enumerate(self.engines):
            self.send[k].ensure(sum(sizes[k]))
            e.wire_pack(self.send[k].ptr(), self.send[k].cap())
        for e in self.engines:
            e.sync()
        self.wire_bytes = sum(sizes[a][b] for a in range(self.N) for b in range(self.N) if a != b)
        for k in range(self.N):
            rs = [sizes[a][k] for a in range(self.N)]
            dst = self.recv[k].ensure(sum(rs))
            pos = 0
            for a in range(self.N):
                n = rs[a]
                if n:
                    so = sum(sizes[a][:k])
                    dst[pos:pos + n].copy_(self.send[a].t[so:so + n])
                pos += n
        torch.cuda.synchronize()
        for k, e in enumerate(self.engines):
            e.wire_recv(self.recv[k].ptr(), [sizes[a][k] for a in range(self.N)])

    def tick(self, prop_target=None, prop_count=None, campaign=None, isolate=None, flags=0, threads=None):
        self.exchange()
        for e in self.engines:
            e.tick(prop_target, prop_count, campaign, isolate, flags)

    @property
    def t(self) -> int:
        return self.engines[0].t

    # ---- views in global ids
    def replicas(self, first=0, n=None):
        n = self.nrep - first if n is None else n
        per = [e.replicas() for e in self.engines]
        return [per[self.loc[r][0]][self.loc[r][1]] for r in range(first, first + n)]

    def replica(self, rid) -> dict:
        k, lr = self.loc[rid]
        return self.engines[k].replica(lr)

    def msgs(self, rid, dst) -> list:
        k, lr = self.loc[rid]
        return self.engines[k].msgs(lr, dst)

    def entries(self, rid, first, n, with_payload=False):
        k, lr = self.loc[rid]
        return self.engines[k].entries(lr, first, n, with_payload)

    def entry(self, rid, index, with_payload=False):
        k, lr = self.loc[rid]
        return self.engines[k].entry(lr, index, with_payload)

    def import_replica(self, rid, view, terms, types=None, payloads=None):
        k, lr = self.loc[rid]
        self.engines[k].import_replica(lr, view, terms, types, payloads)

    def deliver(self, rid_src, **fields):
        k, lr = self.loc[rid_src]
        self.engines[k].deliver(lr, **fields)

    def leader(self, group):
        """NodeHost.GetLeaderID as the node hosting slot 0 of the group sees it."""
        return self.engines[rank_of(group, 0, self.N)].leader(group)

    def sum_committed(self) -> int:
        return sum(e.sum_committed() for e in self.engines)
