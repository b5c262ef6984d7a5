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

import numpy as np

from .engine import Engine, default_config


# ---------------------------------------------------------------- placement (raftgpu_internal.h)
def slot_offset(s: int, j: int, n: int) -> int:
    """off_c(s): rank offset of slot s in column j (class c = j mod (n - 1)); 0 for slot 0."""
    if s == 0 or n < 2:
        return 0
    m, p = n - 1, (s - 1) % n
    if p == m:  # n < R: every n-th follower shares the leader's rank (fewer copies over xGMI)
        return 0
    return (j % m + p) % m + 1


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
# Largest piece of one peer region moved by a single RCCL call. RCCL 2.26.6 (the one bundled with
# this PyTorch) corrupted all_to_all_single regions above 1 GiB: from the region's midpoint on, the
# received bytes were wrong, with no error raised (scripts/a2a_probe.py, one rank, 1100 and 1500 MB;
# exact up to 1024 MB). At N = 2 a rank's whole follower traffic, ~2.3 GB a tick at 64K groups, goes
# to its one peer, so every exchange is cut into calls of at most this many bytes per peer region.
A2A_CHUNK = 256 << 20


class _Works:
    """Work handles of one chunked exchange: wait() orders the current stream after all of them."""

    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()


def a2a_chunks(max_region: int, chunk: int = A2A_CHUNK) -> int:
    return max(1, -(-max_region // chunk))


def all_to_all_bytes(send, send_sizes, recv, recv_sizes, group=None, async_op=False, nchunks=1,
                     chunk=A2A_CHUNK):
    """Move region r of `send` (sizes send_sizes, concatenated in rank order) to rank r; the
    regions from every rank land concatenated in rank order in `recv`. nccl: device tensors moved
    by RCCL over xGMI — one all_to_all_single, or, when a region exceeds `chunk` bytes, `nchunks`
    all_to_all calls over views of at most `chunk` bytes per region (nchunks must be the same on
    every rank: a2a_chunks of the largest region of the exchange); async_op returns a handle whose
    wait() makes the current stream wait. gloo: staged through host memory, always synchronous
    (returns None)."""
    import torch.distributed as dist
    torch = _torch()
    stot, rtot = sum(send_sizes), sum(recv_sizes)
    if dist.get_backend(group) == "nccl":
        if nchunks <= 1:
            return dist.all_to_all_single(recv[:rtot], send[:stot], list(recv_sizes), list(send_sizes), group=group,
                                          async_op=async_op)
        so, _ = _offsets(send_sizes)
        ro, _ = _offsets(recv_sizes)
        works = []
        for k in range(nchunks):
            lo, hi = k * chunk, (k + 1) * chunk
            ins = [send[so[r] + min(lo, n):so[r] + min(hi, n)] for r, n in enumerate(send_sizes)]
            outs = [recv[ro[r] + min(lo, n):ro[r] + min(hi, n)] for r, n in enumerate(recv_sizes)]
            works.append(dist.all_to_all(outs, ins, group=group, async_op=True))
        h = _Works(works)
        if async_op:
            return h
        h.wait()
        return None
    hs = send[:stot].cpu() if send.is_cuda else send[:stot]
    hr = torch.empty(rtot, dtype=torch.uint8)
    dist.all_to_all_single(hr, hs, list(recv_sizes), list(send_sizes), group=group)
    recv[:rtot].copy_(hr)
    return None


def p2p_regions(send, send_sizes, recv, recv_sizes, group=None, async_op=False, chunk=A2A_CHUNK, send_offs=None,
                self_p2p=False):
    """The exchange's transfer on nccl, fixed or exactly sized: region r of `send` to rank r and region
    r of `recv` from rank r as one batch of point-to-point sends and receives (one grouped RCCL call),
    each piece at most `chunk` bytes (the 1 GiB contract). A link's two ends agree on its size, so
    they cut it into the same pieces without any rank knowing the others' sizes (an all_to_all's
    chunk count has to be the same on every rank). The region to this rank itself is a device copy.
    send_offs: the send regions' offsets in `send` when not consecutive (a region of 0 bytes to this
    rank: it was packed in place, nothing to copy). self_p2p (tests): the region to this rank goes through
    the same point-to-point pieces as the others, so a one-rank group runs the grouped path.
    nccl only; gloo ranks go through all_to_all_bytes."""
    import torch.distributed as dist
    me, n = dist.get_rank(group), dist.get_world_size(group)
    so = list(send_offs) if send_offs is not None else _offsets(send_sizes)[0]
    ro, _ = _offsets(recv_sizes)
    if send_sizes[me] and not self_p2p:
        recv[ro[me]:ro[me] + recv_sizes[me]].copy_(send[so[me]:so[me] + send_sizes[me]])
    ops = []
    for r in range(n):
        if r == me and not self_p2p:
            continue
        peer = dist.get_global_rank(group, r) if group is not None else r
        for lo in range(0, send_sizes[r], chunk):
            ops.append(dist.P2POp(dist.isend, send[so[r] + lo:so[r] + min(send_sizes[r], lo + chunk)], peer, group))
        for lo in range(0, recv_sizes[r], chunk):
            ops.append(dist.P2POp(dist.irecv, recv[ro[r] + lo:ro[r] + min(recv_sizes[r], lo + chunk)], peer, group))
    h = _Works(dist.batch_isend_irecv(ops) if ops else [])
    if async_op:
        return h
    h.wait()
    return None


def exchange_sizes(send_sizes, group=None):
    """Each rank's outbound region sizes → (the sizes this rank receives from every rank, the
    largest region any rank sends this exchange), by one all_gather of the size rows."""
    import torch.distributed as dist
    torch = _torch()
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    n = dist.get_world_size(group)
    st = torch.tensor(send_sizes, dtype=torch.int64, device=dev)
    allt = torch.empty(n * len(send_sizes), dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allt, st, group=group)
    m = allt.view(n, len(send_sizes)).tolist()  # m[a][b]: rank a → rank b
    me = dist.get_rank(group)
    return [m[a][me] for a in range(n)], max(max(row) for row in m)


def _dev_bytes(ptr: int, n: int, device):
    """A uint8 torch tensor over n bytes of device memory the engine owns (no copy)."""
    torch = _torch()

    class _Arr:
        __cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False), "version": 3,
                                    "strides": None}

    return torch.as_tensor(_Arr(), device=device) if n else torch.empty(0, dtype=torch.uint8, device=device)


def gloo_transport(pg, device):
    """rg_transport over a gloo (or any host) process group, for rg_wire_exchange: sizes by
    all_gather, regions staged through host memory by all_to_all_bytes. Synchronous: it waits
    for the engine stream before reading and completes before returning (include/raftgpu.h)."""
    import torch.distributed as dist
    from .engine import PyTransport
    torch = _torch()
    n = dist.get_world_size(pg)

    def allgather(vals):
        t = torch.tensor(vals, dtype=torch.int64)
        out = [torch.empty_like(t) for _ in range(n)]
        dist.all_gather(out, t, group=pg)
        return [int(v) for o in out for v in o.tolist()]

    def alltoallv(send, soff, ssize, recv, roff, rsize, stream):
        torch.cuda.synchronize(device)
        ss, rs = [int(ssize[r]) for r in range(n)], [int(rsize[r]) for r in range(n)]
        # the regions sit at the offsets given (rg_wire_exchange packs the region to self in place and
        # the others after the receive regions), staged here in rank order
        sb = torch.cat([_dev_bytes(send + int(soff[r]), ss[r], device) for r in range(n)])
        rb = torch.empty(sum(rs), dtype=torch.uint8, device=device)
        big = torch.tensor([max(ss + rs)], dtype=torch.int64)
        dist.all_reduce(big, op=dist.ReduceOp.MAX, group=pg)  # every rank issues the same chunk count
        all_to_all_bytes(sb, ss, rb, rs, pg, nchunks=a2a_chunks(int(big.item())))
        o = 0
        for r in range(n):
            if rs[r]:
                _dev_bytes(recv + int(roff[r]), rs[r], device).copy_(rb[o:o + rs[r]])
            o += rs[r]
        torch.cuda.synchronize(device)

    pt = PyTransport(allgather, alltoallv)
    pt.nranks = n
    return pt


class _Half:
    """One engine of a rank and its exchange state. start() ships the last tick's cross-rank
    messages (plan, pack, size exchange, all-to-all — asynchronous on nccl); finish() waits for
    them and unpacks before the engine's next tick. With a C transport (exchange="c") start() is
    one rg_wire_exchange call, ordered on the device, and finish() has nothing left to do."""

    def __init__(self, eng, dev, pg, rank, xt=None, fixed=True, p2p_self=False):
        self.eng, self.pg, self.rank, self.xt, self.fixed, self.p2p_self = eng, pg, rank, xt, fixed, p2p_self
        self.send, self.recv = _Buf(dev), _Buf(dev)  # nccl: self.recv holds both (send regions after the receive ones)
        self.work, self.rsizes, self.sent = None, None, 0

    def start(self, async_op):
        e = self.eng
        if self.xt is not None:
            self.sent = e.wire_exchange(self.xt)
            return
        import torch.distributed as dist
        if self.fixed:
            # one grouped transfer, no host sync: capacities both ends of every link agree on (rg_wire_plan_fixed)
            sizes, rsizes = e.wire_plan_fixed()
            biggest = max(sizes + rsizes)  # gloo: host-staged, one call
        else:
            sizes = e.wire_plan()  # host sync: the tick that produced the messages has completed
        _, stot = _offsets(sizes)
        if not self.fixed:
            rsizes, biggest = exchange_sizes(sizes, self.pg)
        ro, rtot = _offsets(rsizes)
        me = self.rank
        if dist.get_backend(self.pg) == "nccl" and sizes[me] and sizes[me] == rsizes[me] and not self.p2p_self:
            # one buffer: the receive regions, then the send regions to the other ranks; the region to
            # this rank is packed where wire_recv reads it (no self copy; rg_wire_pack_at). Stream order:
            # the tick that read the old contents runs before the pack and the transfers
            sbase = (rtot + 255) & ~255
            so, o = [], sbase
            for r, n in enumerate(sizes):
                so.append(ro[r] if r == me else o)
                o += 0 if r == me else n
            self.recv.ensure(max(o, 256))
            e.wire_pack_at(self.recv.ptr(), so, self.recv.cap())
            ssz = list(sizes)
            ssz[me] = 0
            rsz = list(rsizes)
            rsz[me] = 0
            self.work = p2p_regions(self.recv.t, ssz, self.recv.t, rsz, self.pg, async_op=async_op, send_offs=so)
            self.rsizes, self.sent = rsizes, stot - sizes[me]
            return
        self.send.ensure(stot)
        e.wire_pack(self.send.ptr(), self.send.cap())
        self.recv.ensure(rtot)  # stream order: the tick that reads the old buffer runs before a reuse
        if dist.get_backend(self.pg) == "nccl":  # the region to this rank: a device copy, not RCCL
            self.work = p2p_regions(self.send.t, sizes, self.recv.t, rsizes, self.pg, async_op=async_op,
                                    self_p2p=self.p2p_self)
        else:
            self.work = all_to_all_bytes(self.send.t, sizes, self.recv.t, rsizes, self.pg, async_op=async_op,
                                         nchunks=a2a_chunks(biggest))
        self.rsizes, self.sent = rsizes, stot - sizes[self.rank]

    def finish(self):
        if self.work is not None:
            self.work.wait()
            self.work = None
        if self.rsizes is not None:
            self.eng.wire_recv(self.recv.ptr(), self.rsizes)
            self.rsizes = None


class _Feeds:
    """The per-tick host feeds (rg_snapshot_events, rg_apply_committed) over several engines, in
    this object's replica ids, replica order (what SnapshotDriver / Applier consume)."""

    _rid_base = 0

    def _feed_engines(self):
        raise NotImplementedError

    def _feed_maps(self):
        if getattr(self, "_gmaps", None) is None:  # local rid → id here, once
            self._gmaps = [np.array([e.global_id(lr)[1] for lr in range(e.nrep)], np.int64) - self._rid_base
                           for e in self._feed_engines()]
        return self._gmaps

    def snapshot_events(self, slot_mask: int = 0xFF):
        parts = []
        for e, gm in zip(self._feed_engines(), self._feed_maps()):
            ev = e.snapshot_events(slot_mask).copy()
            ev["rid"] = gm[ev["rid"].astype(np.int64)]
            parts.append(ev)
        out = np.concatenate(parts)
        return out[np.argsort(out["rid"], kind="stable")]

    def apply_committed(self, slot_mask: int = 0xFF):
        recs, pays = [], []
        for e, gm in zip(self._feed_engines(), self._feed_maps()):
            r, p = e.apply_committed(slot_mask)
            r = r.copy()
            r["rid"] = gm[r["rid"].astype(np.int64)]
            recs.append(r)
            pays.append(p)
        w = max(p.shape[1] for p in pays)  # row widths follow each engine's batch (engine.row_width)
        pays = [np.pad(p, ((0, 0), (0, w - p.shape[1]))) for p in pays]
        recs, pays = np.concatenate(recs), np.concatenate(pays)
        order = np.argsort(recs["rid"], kind="stable")  # each replica's entries stay in index order
        return recs[order], pays[order]


class DistEngine(_Feeds):
    """This process's share of an N-rank cluster (rank = torch.distributed rank): `groups` local
    columns (the cluster hosts ranks * groups shards), as `halves` engines over disjoint column
    ranges. Engines launch on torch's current stream, so each exchange orders itself behind the
    tick that produced it. With two halves, step_device() pipelines: while one half's all-to-all
    is on the wire, the other half unpacks, ticks and packs."""

    def __init__(self, groups: int, group=None, halves: int = 1, exchange: str = "torch", fixed=None,
                 p2p_self: bool = False, **cfg):
        """exchange: "torch" moves the regions with torch.distributed from Python; "c" with the
        library's rg_wire_exchange (RCCL transport on an nccl group, a host-staged one on gloo),
        each half on a stream of its own so one half's transfer overlaps the other's tick.
        fixed: size the regions with rg_wire_plan_fixed (no host sync, no size exchange: the all-to-all
        is the tick's one collective; a transfer moves each link's capacity, which follows its need,
        DESIGN.md §6) — the default — or, False, with rg_wire_plan (exact sizes after a host sync and a
        size all-gather; on the C exchange through rg_config.wire_exact).
        p2p_self (tests): on nccl the region to this rank goes through the point-to-point pieces like
        every other region, so a one-rank group runs the N > 1 transfer path."""
        import torch.distributed as dist
        torch = _torch()
        if groups % halves:
            raise ValueError("groups must be a multiple of halves")
        if exchange not in ("torch", "c"):
            raise ValueError("exchange is 'torch' or 'c'")
        self.pg = group
        self.N, self.rank = dist.get_world_size(group), dist.get_rank(group)
        hg = groups // halves
        self.cols = hg
        self.fixed = True if fixed is None else bool(fixed)
        cfg = dict(cfg, wire_exact=0 if self.fixed else 1)
        engs = [Engine(groups=hg, ranks=self.N, rank=self.rank, column_base=h * hg, **cfg) for h in range(halves)]
        torch.cuda.set_device(engs[0].cfg["device"])
        self.stream = torch.cuda.current_stream()
        if self.stream.cuda_stream == 0:  # the engine needs a real stream shared with torch's copies
            self.stream = torch.cuda.Stream()
            torch.cuda.set_stream(self.stream)
        dev = torch.device("cuda", engs[0].cfg["device"])
        self.xchg, self.xt, self._xclose = exchange, None, None
        self.streams = [self.stream] + ([torch.cuda.Stream(device=dev) for _ in engs[1:]] if exchange == "c"
                                        else [self.stream] * (len(engs) - 1))
        for e, st in zip(engs, self.streams):
            e.set_stream(st.cuda_stream)
        if exchange == "torch" and dist.get_backend(group) == "nccl":
            # the exchange is a batch of point-to-point sends and receives (p2p_regions); NCCL wants the
            # communicator made by a collective of the whole group first
            dist.barrier(group=group)
        if exchange == "c":
            from .engine import rccl_close, rccl_transport, rccl_unique_id
            if dist.get_backend(group) == "nccl":
                uid = [rccl_unique_id() if self.rank == 0 else None]
                dist.broadcast_object_list(uid, src=0, group=group)
                t = rccl_transport(uid[0], self.N, self.rank, engs[0].cfg["device"])
                self.xt, self._xclose = t, (lambda: rccl_close(t))
            else:
                self._pyxt = gloo_transport(group, dev)
                self.xt = self._pyxt.t
        self.parts = [_Half(e, dev, self.pg, self.rank, self.xt, fixed=self.fixed, p2p_self=p2p_self) for e in engs]
        self.eng = engs[0]
        self.cfg, self.R = engs[0].cfg, engs[0].R
        self.async_ok = dist.get_backend(group) == "nccl"
        self.primed = False

    def _feed_engines(self):  # host feeds in global replica ids
        self.drain()
        return [p.eng for p in self.parts]

    @property
    def wire_bytes(self) -> int:  # bytes this rank sent in the last exchange of every half
        return sum(p.sent for p in self.parts)

    def _slices(self, h):
        """Offsets of half h's tick inputs in the global arrays: groups, replicas."""
        g0 = self.N * self.cols * h
        return g0, g0 * self.R

    # ---- plain (exchange, then tick): bring-up, tests
    def exchange(self):
        for p in self.parts:
            p.start(async_op=False)
            p.finish()

    def tick(self, prop_target=None, prop_count=None, campaign=None, isolate=None, flags=0):
        self.drain()
        n = self.N * self.cols
        for h, p in enumerate(self.parts):
            p.start(async_op=False)
            p.finish()
            g0, r0 = self._slices(h)
            sl = lambda a, o, k: None if a is None else a[o:o + k]  # noqa: E731
            p.eng.tick(sl(prop_target, g0, n), sl(prop_count, g0, n), sl(campaign, r0, n * self.R),
                       sl(isolate, r0, n * self.R), flags)

    def tick_device(self, pt_ptr=0, pc_ptr=0, flags=0):
        self.drain()
        for h, p in enumerate(self.parts):
            p.start(async_op=False)
            p.finish()
            g0, _ = self._slices(h)
            p.eng.tick_device(pt_ptr + g0 if pt_ptr else 0, pc_ptr + 4 * g0 if pc_ptr else 0, flags=flags)

    # ---- pipelined steady state (device-resident proposal inputs)
    def prime(self):
        """Start every half's exchange of its last tick (before the first step_device)."""
        if not self.primed:
            for p in self.parts:
                p.start(async_op=self.async_ok)
            self.primed = True

    def step_device(self, pt_ptr=0, pc_ptr=0, flags=0, persist=None):
        """One pipelined step. persist(engine), if given, runs after each half's tick and before
        that tick's messages are packed and leave the rank: the place for rg_persist_collect + WAL
        fsync (dragonboat persists a step's Update before its messages go out). Without
        it this path is not durable (the benchmark's mode)."""
        self.prime()
        for h, p in enumerate(self.parts):
            p.finish()
            g0, _ = self._slices(h)
            p.eng.tick_device(pt_ptr + g0 if pt_ptr else 0, pc_ptr + 4 * g0 if pc_ptr else 0, flags=flags)
            if persist is not None:
                persist(p.eng)
            p.start(async_op=self.async_ok)

    def drain(self):
        """Complete the exchanges in flight so every engine is ready for a plain tick or a read."""
        if self.primed:
            for p in self.parts:
                p.finish()
            self.primed = False

    # ---- caller inputs in global shard ids, routed to the half hosting the shard's column; the
    # replicas other ranks host are theirs to stage (every rank may pass the same list)
    def _half_engine(self, group: int):
        return self.parts[(group // self.N) // self.cols].eng

    def hosts(self, group: int, slot: int) -> bool:
        """Whether this rank hosts replica `slot` of global shard `group` (placement)."""
        return rank_of(group, slot, self.N) == self.rank

    def _local(self, group: int, slot: int):
        """(half engine, its local replica id) of replica `slot` of global shard `group` (hosted here)."""
        if not self.hosts(group, slot):
            raise ValueError(f"replica {slot} of shard {group} is hosted by rank {rank_of(group, slot, self.N)}")
        j = group // self.N
        h = j // self.cols
        return self.parts[h].eng, (j - h * self.cols) * self.R + slot

    def replica_of(self, group: int, slot: int) -> dict:
        """rg_read_replicas of replica `slot` of global shard `group` (hosted by this rank)."""
        self.drain()
        e, rid = self._local(group, slot)
        return e.replica(rid)

    def import_replica_of(self, group: int, slot: int, view, terms, types=None, payloads=None, lens=None):
        """rg_import_replica of replica `slot` of global shard `group` (hosted by this rank)."""
        self.drain()
        e, rid = self._local(group, slot)
        e.import_replica(rid, view, terms, types, payloads, lens)

    @property
    def t(self) -> int:
        return self.eng.t

    def propose(self, batches):
        """rg_propose of the batches [(global group, slot, [Cmd bytes])] whose replica is hosted here."""
        per = {}
        for g, s, cmds in batches:
            if self.hosts(g, s):
                e = self._half_engine(g)
                per.setdefault(id(e), (e, []))[1].append((g, s, cmds))
        for e, b in per.values():
            e.propose(b)

    def config_change(self, group, slot, op, target):
        """rg_config_change, if replica `slot` of global shard `group` is hosted here."""
        if self.hosts(group, slot):
            self._half_engine(group).config_change(group, slot, op, target)

    def read_index(self, reqs):
        """rg_read_index of the requests [(global group, slot, ctx)] whose replica is hosted here."""
        per = {}
        for g, s, ctx in reqs:
            if self.hosts(g, s):
                e = self._half_engine(g)
                per.setdefault(id(e), (e, []))[1].append((g, s, ctx))
        for e, b in per.values():
            e.read_index(b)

    # ---- aggregates over the halves (bench)
    def bootstrap(self):
        for p in self.parts:
            p.eng.bootstrap()

    def join(self):
        """torch's current stream waits (on the device) for every half's last tick."""
        torch = _torch()
        cur = torch.cuda.current_stream()
        for p, st in zip(self.parts, self.streams):
            p.eng.join()
            if st.cuda_stream != cur.cuda_stream:
                ev = torch.cuda.Event()
                ev.record(st)
                cur.wait_event(ev)

    def sync(self):
        for p in self.parts:
            p.eng.sync()

    def close(self):
        """Release the RCCL communicator of exchange="c" (after the last exchange completed)."""
        self.sync()
        if self._xclose is not None:
            self._xclose()
            self._xclose, self.xt = None, None

    def timing(self, on=True, bulk_only=False, every=1):
        for p in self.parts:
            p.eng.timing(on, bulk_only=bulk_only, every=every)

    def kernel_ms(self) -> dict:
        """Summed over the halves: total ms per kernel, and launches counted per tick."""
        ks = [p.eng.kernel_ms() for p in self.parts]
        return {k: (sum(x[k][0] for x in ks), ks[0][k][1]) for k in ks[0]}

    def kernel_span_ms(self, kernel: str = "bulk"):
        """The kernel's wall-clock time per tick over the halves — the union of the halves' launch
        intervals of the same tick on the epoch timeline (rg_timing_epoch before timing(True)) — summed
        over the ticks every half timed, and their count. Halves on streams of their own overlap, so the
        sum of their launch durations overstates the time the tick spent in the kernel; halves on one
        stream run other work between their launches, so a first-start-to-last-end span would overstate
        it too; the union does neither."""
        per = {}
        for p in self.parts:
            ticks, a, b = p.eng.kernel_events(kernel)
            for t, x, y in zip(ticks.tolist(), a.tolist(), b.tolist()):
                per.setdefault(t, []).append((x, y))
        out = []
        for v in per.values():
            if len(v) != len(self.parts):
                continue
            tot, end = 0.0, None
            for x, y in sorted(v):
                if end is None or x > end:
                    tot += y - x
                    end = y
                elif y > end:
                    tot += y - end
                    end = y
            out.append(tot)
        return sum(out), len(out)

    def last_tick_traffic(self) -> dict:
        ts = [p.eng.last_tick_traffic() for p in self.parts]
        return {k: sum(t[k] for t in ts) for k in ts[0]}

    def sum_committed(self) -> int:
        return sum(p.eng.sum_committed() for p in self.parts)

    @property
    def device_bytes(self) -> int:
        return sum(p.eng.device_bytes for p in self.parts)


# ---------------------------------------------------------------- N ranks in one process
class LoopbackCluster(_Feeds):
    """N engines (ranks) in one process on one GPU, moving regions with device copies. The
    interface is the single Engine's, in global ids counted from the cluster's first group
    (ranks * column_base, like an oracle window's group_base): replica id g * R + s, `groups` =
    all ranks' shards (a multiple of ranks)."""

    def __init__(self, ranks: int, groups: int, column_base: int = 0, **cfg):
        torch = _torch()
        if groups % ranks:
            raise ValueError("groups must be a multiple of ranks")
        self.N = ranks
        self.cfg = default_config(groups=groups, **cfg)
        self.G, self.R = groups, self.cfg["replicas"]
        self.nrep = self.G * self.R
        self.rid0 = ranks * column_base * self.R  # ids are relative to the first group, as inputs are
        self._rid_base = self.rid0
        lc = dict(self.cfg, groups=groups // ranks, column_base=column_base)
        self.engines = [Engine(**dict(lc, ranks=ranks, rank=k)) for k in range(ranks)]
        dev = torch.device("cuda", self.cfg["device"])
        self.send = [_Buf(dev) for _ in range(ranks)]
        self.recv = [_Buf(dev) for _ in range(ranks)]
        self.loc = [None] * self.nrep  # global rid → (rank, local rid)
        for k, e in enumerate(self.engines):
            for lr in range(e.nrep):
                g, gr = e.global_id(lr)
                self.loc[gr - self.rid0] = (k, lr)
        self.wire_bytes = 0
        self.on_recv = None  # callable(rank, recv tensor, region sizes) before unpack (tests)

    def close(self):
        for e in self.engines:
            e.close()

    def _feed_engines(self):
        return self.engines

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
        if self.on_recv is not None:  # tests: inspect or damage the received regions
            for k in range(self.N):
                self.on_recv(k, self.recv[k].t, [sizes[a][k] for a in range(self.N)])
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

    @property
    def device_bytes(self) -> int:
        return sum(e.device_bytes for e in self.engines)

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

    def import_replica(self, rid, view, terms, types=None, payloads=None, lens=None):
        k, lr = self.loc[rid]
        self.engines[k].import_replica(lr, view, terms, types, payloads, lens)

    def notify_applied(self, rids, index):
        """rg_notify_applied on the ranks hosting replicas rids (cluster ids)."""
        for r, i in zip(np.atleast_1d(rids), np.atleast_1d(index)):
            k, lr = self.loc[int(r)]
            self.engines[k].notify_applied([lr], [int(i)])

    def config_change(self, group, slot, op, target):
        """rg_config_change on the rank hosting replica `slot` of cluster group `group`."""
        gg = group + self.rid0 // self.R
        self.engines[rank_of(gg, slot, self.N)].config_change(gg, slot, op, target)

    def read_index(self, reqs):
        """rg_read_index on the rank hosting each request's replica (cluster group ids)."""
        per = [[] for _ in range(self.N)]
        for g, s, ctx in reqs:
            gg = g + self.rid0 // self.R
            per[rank_of(gg, s, self.N)].append((gg, s, ctx))
        for k, b in enumerate(per):
            if b:
                self.engines[k].read_index(b)

    def read_ready_all(self) -> dict:
        """{cluster rid: [(ctx, index), ...]} for the reads made ready in the last tick, over all ranks."""
        back = {kl: r for r, kl in enumerate(self.loc)}
        out = {}
        for k, e in enumerate(self.engines):
            for lr, v in e.read_ready_all().items():
                out[back[(k, lr)]] = v
        return out

    def read_ready(self, rid):
        """[(ctx, index), ...] made ready for cluster replica rid in the last tick."""
        return self.read_ready_all().get(rid, [])

    def propose(self, batches):
        """rg_propose on the rank hosting each batch's replica (global group, slot)."""
        per = [[] for _ in range(self.N)]
        for g, s, cmds in batches:
            gg = g + self.rid0 // self.R  # global group
            per[rank_of(gg, s, self.N)].append((gg, s, cmds))
        for k, b in enumerate(per):
            if b:
                self.engines[k].propose(b)

    def deliver(self, rid_src, **fields):
        k, lr = self.loc[rid_src]
        self.engines[k].deliver(lr, **fields)

    def rank_view(self, rank: int) -> "RankView":
        """Rank `rank`'s share of this cluster, with a per-rank NodeHost's interface (tests: several
        NodeHosts over one LoopbackCluster, the driver ticking the cluster once per tick)."""
        return RankView(self, rank, self.N, self.R)

    def leader(self, group):
        """NodeHost.GetLeaderID as the node hosting slot 0 of the group sees it."""
        return self.engines[rank_of(group, 0, self.N)].leader(group)

    def sum_committed(self) -> int:
        return sum(e.sum_committed() for e in self.engines)


class RankView:
    """One rank's share of a whole-cluster backend (LoopbackCluster, or the oracle of every shard in
    tests): the replicas `rank` hosts under the spread placement, addressed by (global shard, slot),
    as raftd_amd.nodehost.NodeHost uses them. tick() is the backend's, which the driver calls once
    per tick for all ranks (NodeHost.before_tick / after_tick around it)."""

    def __init__(self, backend, rank: int, ranks: int, replicas: int):
        self.b, self.rank, self.N, self.R = backend, rank, ranks, replicas

    def hosts(self, group: int, slot: int) -> bool:
        return rank_of(group, slot, self.N) == self.rank

    def _rid(self, group: int, slot: int) -> int:
        if not self.hosts(group, slot):
            raise ValueError(f"replica {slot} of shard {group} is not hosted by rank {self.rank}")
        return group * self.R + slot

    def replica_of(self, group: int, slot: int) -> dict:
        return self.b.replica(self._rid(group, slot))

    def import_replica_of(self, group: int, slot: int, view, terms, types=None, payloads=None, lens=None):
        self.b.import_replica(self._rid(group, slot), view, terms, types, payloads, lens)

    def config_change(self, group: int, slot: int, op: int, target: int):
        self._rid(group, slot)
        rc = self.b.config_change(group, slot, op, target)
        if rc not in (None, 0):
            raise RuntimeError(f"config_change({group}, {slot}, {op}, {target}): {rc}")

    @property
    def t(self) -> int:
        t = getattr(self.b, "t", None)
        return t if t is not None else self.b.tick_count()
