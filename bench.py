"""raftd-amd benchmark: batched Raft group-steps/s and commits/s on MI355X.

Workload (BASELINE.json metric "raft group-steps/sec & commits/sec, 64K groups x 3 replicas"):
65,536 Raft groups x 3 replicas per GPU, steady state (slot 0 leads each group after a real
election through the engine), every tick each leader receives a 64-entry proposal batch of
256-B payloads (CRC32 per entry at every replica), raftd's Raft config (ElectionRTT 10,
HeartbeatRTT 1, CheckQuorum, SnapshotEntries 1000, CompactionOverhead 5). A step = one tick of
every replica of every group = one control_kernel launch (Raft logic) + one bulk_kernel launch
(payload copies + CRC32), in that order on one stream. Inputs (proposal descriptors, payload
slabs) are resident in HBM before the timed region.

roofline: the dominant kernel is bulk_kernel (HBM-bound byte copies + CRC). achieved = its
algorithmic bytes per launch (rg_traffic.bulk_bytes) / its mean launch duration, timed with HIP
events recorded on the engine stream around every launch of the timed region. With
--payload 0 there is no payload stage and the control kernel (the whole tick's algorithmic bytes)
is reported instead.

N > 1 (default --placement spread, the north star's layout): one process per GPU
(torch.distributed.run), N x 65,536 groups, replica slot s of group g on GPU (g mod N + off(s)) mod N
(DESIGN.md §6), so every replica of a group sits on a different GPU, emulating separate nodes.
Each step = the exchange of the previous tick's cross-GPU messages (plan/pack kernels, one grouped
RCCL send/recv per peer over xGMI — an all-to-all, the only collective — and the unpack kernel) + the
tick (the line's `parallelism` / exchange.transport name the transport that ran); with
--halves 2 (default) each GPU's columns are two engines whose exchanges are pipelined behind each
other's ticks. Every GPU
hosts 196,608 replicas, as at N = 1 (weak scaling). --placement colocated keeps every replica of
a group on one GPU (no exchange). value = groups over all ranks x K / max-over-ranks time.
--wire-all (N = 1, measurement): every message goes through the pack/unpack path to itself.

Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time


ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "raft group-steps/sec & commits/sec, 64K groups×3 replicas, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
XGMI_LINK_GBS = 153.0  # one xGMI link per GPU pair, 7 per GPU (≈153 GB/s each)
CONTROL_TIMING_STEPS = 4
TIMING_EVERY = 4  # bulk_kernel launches timed with events: one tick in four of the timed region


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--groups", type=int, default=65536)
    ap.add_argument("--replicas", type=int, default=3)
    ap.add_argument("--entries", type=int, default=64)
    ap.add_argument("--payload", type=int, default=256)
    ap.add_argument("--log-capacity", type=int, default=2048)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--placement", choices=["spread", "colocated"], default=None,
                    help="N > 1: replicas of a group on different GPUs (default) or on one")
    ap.add_argument("--wire-all", action="store_true", help="N = 1: route every message through the wire; with "
                    "--placement spread, through the N > 1 code path (DistEngine, halves, RCCL all-to-all to "
                    "itself in a one-rank process group): a rehearsal of the multi-GPU step on one GPU")
    ap.add_argument("--halves", type=int, default=2, help="N > 1 spread: engines per rank over disjoint column "
                    "ranges; 2 pipelines one half's all-to-all behind the other half's tick (1 = no overlap)")
    ap.add_argument("--sizing", choices=["exact", "fixed"], default=None,
                    help="spread placement, either exchange: region sizing (default fixed: the all-to-all is the "
                         "tick's one collective; exact: a plan host sync and a size all-gather first; DESIGN.md §6)")
    ap.add_argument("--exchange", choices=["torch", "c"], default="torch", help="N > 1 spread: move the regions "
                    "with torch.distributed from Python (default) or with the library's rg_wire_exchange (built-in "
                    "RCCL transport on nccl; each half on its own stream)")
    ap.add_argument("--ingest", action="store_true", help="N = 1: also time the client ingest path: every step "
                    "the G x E Cmds enter through rg_propose from host memory (NodeHost.Propose) instead of the "
                    "HBM-resident proposal slabs; reported beside the headline line as `ingest`")
    ap.add_argument("--backend", default="nccl", help="N > 1: nccl (RCCL, default) or gloo (rehearsal: several "
                    "ranks on one GPU with RAFTD_BENCH_DEVICE=0, regions staged through host memory)")
    ap.add_argument("--dry-run", action="store_true", help="N > 1 launcher check: every rank joins the process "
                    "group on the CPU (gloo), agrees on the world size and exits without touching a GPU")
    return ap.parse_args()


def exchange_transport(spread: bool, wire_all: bool, exchange: str, backend: str, fixed: bool):
    """How the N > 1 step moves its regions, in the words the line's `parallelism` label and
    `exchange.transport` both use (the label must name the transport that actually ran)."""
    if not spread:
        return "device copy (one engine)" if wire_all else None
    sizing = ("fixed-capacity regions (no host sync, no size exchange)" if fixed
              else "exactly sized regions (plan host sync + size all-gather)")
    if exchange == "c":
        how = ("rg_wire_exchange (C-ABI) with its built-in RCCL transport: one grouped ncclSend / ncclRecv per peer"
               if backend == "nccl" else "rg_wire_exchange (C-ABI) over a host-staged gloo transport")
    else:
        how = ("torch.distributed batch_isend_irecv: one grouped RCCL send / recv per peer" if backend == "nccl"
               else "torch.distributed all_to_all over gloo, staged through host memory")
    return f"{how}, {sizing}"


def xgmi_bound_ms(bytes_per_step_max_rank: float, world: int):
    """The per-tick floor the exchange puts on an N-GPU step: the busiest rank's outbound bytes over its
    N - 1 direct xGMI links (one per peer on an 8-GPU node, XGMI_LINK_GBS each way), the placement
    spreading a rank's traffic evenly over its peers. None at N = 1 (no link)."""
    if world < 2:
        return None
    return bytes_per_step_max_rank / (min(world - 1, 7) * XGMI_LINK_GBS * 1e9) * 1e3


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """`bench.py --gpus N` started as ONE process (N > 1, no WORLD_SIZE in the environment): start N
    fresh child processes of this script, rank r on GPU r (with --backend gloo every rank on GPU 0: the
    one-GPU rehearsal), rendezvous on 127.0.0.1. This parent makes no GPU call (torch.cuda.device_count
    does not initialise the device on this image) and never execs: it forwards rank 0's JSON line and
    exits non-zero if any rank fails (the others are then stopped). Under torch.distributed.run, the
    driver's N > 1 launcher, every process is already a rank and this is not used."""
    import signal
    import subprocess
    n = args.gpus
    if not args.dry_run:
        import torch
        visible = torch.cuda.device_count()
        if n > visible and args.backend != "gloo":
            print(f"bench.py: --gpus {n} but {visible} GPU(s) visible; use --backend gloo to rehearse {n} ranks "
                  f"on one GPU", file=sys.stderr)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RAFTD_BENCH_CHILD="1")
        if args.backend == "gloo" and not args.dry_run:
            env["RAFTD_BENCH_DEVICE"] = env.get("RAFTD_BENCH_DEVICE", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else None, start_new_session=True))
    import threading
    chunks = []
    reader = threading.Thread(target=lambda: chunks.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    rc = 0
    while any(p.poll() is None for p in procs):
        failed = [p for p in procs if p.returncode not in (None, 0)]
        if failed:  # a failed rank leaves the others waiting in a collective forever: stop them
            rc = failed[0].returncode
            for p in procs:
                if p.poll() is None:
                    os.killpg(p.pid, signal.SIGTERM)
            break
        time.sleep(0.2)
    for p in procs:
        p.wait()
        rc = rc or p.returncode
    reader.join()
    sys.stdout.write(b"".join(chunks).decode())
    sys.stdout.flush()
    return 1 if rc else 0


def dry_run(args, rank, world):
    """The launcher's check (CPU only): join a gloo group, agree on the world size, print the line rank 0
    would carry, exit."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([1.0])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "dry_run": True, "n_gpus": dist.get_world_size(),
                          "ranks_agreeing": int(t.item()), "backend": args.backend}), flush=True)
    dist.destroy_process_group()


def bring_up(eng, tick, G, R):
    """bootstrap → tick → campaign slot 0 → election completes. G = global groups."""
    import numpy as np
    eng.bootstrap()
    tick()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    tick(campaign=camp)
    for _ in range(4):
        tick()


class SelfWire:
    """N = 1 with wire_all: the one region goes to this rank itself (no copy: recv = send)."""

    def __init__(self, eng, torch):
        self.eng, self.torch, self.buf = eng, torch, None
        self.wire_bytes = 0

    def exchange(self):
        sizes, rsizes = self.eng.wire_plan_fixed()  # fixed capacity: no host sync
        n = sum(sizes)
        if self.buf is None or self.buf.numel() < n:
            self.eng.sync()
            self.buf = self.torch.empty(max(n, 1 << 20) * 3 // 2, dtype=self.torch.uint8, device="cuda")
        self.eng.wire_pack(self.buf.data_ptr(), self.buf.numel())
        self.eng.wire_recv(self.buf.data_ptr(), rsizes)
        self.wire_bytes = n

    def tick(self, *a, **kw):
        self.exchange()
        self.eng.tick(*a, **kw)

    def tick_device(self, *a, **kw):
        self.exchange()
        self.eng.tick_device(*a, **kw)


def cpu_baseline(args, seconds):
    """The C oracle (restatement of dragonboat's step) on host threads, dragonboat's step-worker
    arrangement (group g → worker g % T), same per-group workload, bounded sample."""
    import numpy as np
    from oracle.pyoracle import Oracle

    G, R, E = 2048, args.replicas, args.entries
    try:
        T = min(16, len(os.sched_getaffinity(0)))
    except AttributeError:
        T = min(16, os.cpu_count() or 1)
    o = Oracle(groups=G, replicas=R, payload_bytes=args.payload, max_entries_per_msg=E,
               log_capacity=args.log_capacity)
    o.bootstrap()
    o.tick(threads=T)
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    o.tick(campaign=camp, threads=T)
    for _ in range(4):
        o.tick(threads=T)
    pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
    warm = max(8, args.log_capacity // E + 8)  # wrap the log ring once
    for _ in range(warm):
        o.tick(pt, pc, threads=T)
    c0 = o.replica(0)["committed"]
    ticks, t0 = 0, time.perf_counter()
    while True:
        o.tick(pt, pc, threads=T)
        ticks += 1
        el = time.perf_counter() - t0
        if el >= seconds and ticks >= 5:
            break
    c1 = o.replica(0)["committed"]
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
    except OSError:
        pass
    return {
        "value": G * ticks / el,
        "unit": "group-steps/s",
        "cores": T,
        "nproc": os.cpu_count(),
        "affinity_cpus": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
        "cpu_model": model,
        "kind": "port",
        "sample": f"{G} groups x {R} replicas, {E} x {args.payload}-B entries per group-tick, {ticks} timed ticks "
                  f"after {warm} warm ticks ({el:.1f} s); C restatement of dragonboat's step (oracle/oracle.c)",
        "commits_per_sec": (c1 - c0) * G / el,
    }


def hbm_copy_ceiling(eng, nbytes=2 << 30, reps=10):
    """This box's streaming-copy rate (read + write bytes / s, rg_probe_copy: 16 B per lane,
    non-temporal, the bulk kernel's access shape): context for the roofline, which is priced
    against the 8 TB/s spec; MI355X boxes differ by ~10% run to run."""
    import ctypes as C
    g = C.c_double()
    rc = eng.L.rg_probe_copy(eng.cfg["device"], nbytes, reps, C.byref(g))
    return g.value if rc == 0 else None


def apply_copyback(eng, torch, slot_mask=1):
    """rg_apply_committed after the last timed tick: the entries the node hosting the slot-0
    replicas hands to /UpdateEntries, gathered on the device as runs (a 48-B head per run of
    consecutive indices, 8 B of {len, crc} per entry) plus the packed Cmds, and copied back into
    engine-owned pinned memory. Host wall time of the whole call (count + scan + gather + D2H + sync)."""
    import ctypes as C
    from raftd_amd.engine import ApplyBatch
    b = ApplyBatch()
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        rc = eng.L.rg_apply_committed(eng.h, slot_mask, C.byref(b))
        dt = time.perf_counter() - t0
        if rc < 0:
            return None
        best = dt if best is None else min(best, dt)
    if not b.n_entries:
        return None
    nb = batch_bytes(b)
    return {"slot_mask": slot_mask, "entries": b.n_entries, "runs": b.n_runs, "bytes": nb, "ms": best * 1e3,
            "GBps": nb / best / 1e9,
            "note": "count + scan + gather kernels (runs + {len, crc} per entry + Cmds packed at their own "
                    "length), then one hipMemcpyAsync into pinned host memory"}


def batch_bytes(b) -> int:
    """Bytes an rg_apply_batch moves over PCIe: run heads, {len, crc} per entry, Cmds (16-B aligned)."""
    a16 = lambda x: (x + 15) // 16 * 16  # noqa: E731
    return a16(b.n_runs * 48) + a16(b.n_entries * 8) + b.payload_bytes


def e2e_with_apply(eng, tick, G, steps, slot_mask=1, serial=False):
    """Ticks with the committed-entry copy-back the daemon needs for /UpdateEntries: after every tick
    rg_apply_async gathers the slot-0 replicas' applied entries (one node's share) and starts their
    D2H copy on the copy stream, double-buffered, so copies overlap the next ticks; the host waits
    for each tick's copy one tick later. Bounded by min(tick rate, PCIe rate)."""
    import torch
    n = nb = 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()

    def done(buf):
        runs, cmds, pk = eng.apply_wait(buf, copy=False)
        return len(cmds), ((len(runs) * 48 + 15) // 16 + (len(cmds) * 8 + 15) // 16) * 16 + pk.size

    for i in range(steps):
        tick()
        eng.apply_async(slot_mask, i & 1)
        if serial:  # the copy completes before the next tick is issued
            a, b = done(i & 1)
            n, nb = n + a, nb + b
        elif i:
            a, b = done((i - 1) & 1)
            n, nb = n + a, nb + b
    if not serial:
        a, b = done((steps - 1) & 1)
        n, nb = n + a, nb + b
    el = time.perf_counter() - t0
    return {"value": G * steps / el, "unit": "group-steps/s", "steps": steps, "ms_per_step": el * 1e3 / steps,
            "entries_per_step": n / steps, "bytes_per_step": nb / steps, "pcie_GBps": nb / el / 1e9,
            "slot_mask": slot_mask, "schedule": "serial" if serial else "overlapped",
            "note": "tick + gather of the applied entries of one node (slot-0 replicas) + D2H into pinned memory "
                    "on a copy stream (rg_apply_async / rg_apply_wait), "
                    + ("waited for before the next tick" if serial else "overlapped with the next tick")
                    + "; PCIe-bound at full batches"}


def copyback_schedules(eng, tick, G, steps, slot_mask=1):
    """The copy-back schedules of DESIGN.md §7, measured warm and in both orders: one warm run grows
    both apply buffers (device staging and pinned host memory) before anything is timed, then serial,
    overlapped, overlapped, serial. The headline is the faster schedule (the mean of its two runs);
    every run is listed, so an order effect shows as a gap between a schedule's two runs."""
    e2e_with_apply(eng, tick, G, steps=2)  # warm: both buffers grow here, outside the timed runs
    runs = []
    for serial in (True, False, False, True):
        r = e2e_with_apply(eng, tick, G, steps=steps, serial=serial, slot_mask=slot_mask)
        runs.append({k: r[k] for k in ("schedule", "ms_per_step", "pcie_GBps")})
    mean = {sch: sum(x["ms_per_step"] for x in runs if x["schedule"] == sch) / 2 for sch in ("serial", "overlapped")}
    best = min(mean, key=mean.get)
    out = e2e_with_apply(eng, tick, G, steps=steps, serial=best == "serial", slot_mask=slot_mask)
    out.update(ms_per_step=mean[best], value=G / (mean[best] / 1e3),
               pcie_GBps=out["bytes_per_step"] / (mean[best] / 1e3) / 1e9,
               schedules_ms_per_step=mean, runs=runs,
               order_spread={sch: abs(runs[0 if sch == "serial" else 1]["ms_per_step"] -
                                      runs[3 if sch == "serial" else 2]["ms_per_step"]) / mean[sch]
                             for sch in mean},
               note=out["note"] + "; headline = the faster schedule, mean of its two runs (warm, both orders)")
    return out


def hand_off(eng, tick, G, steps, slot_mask=1):
    """Ticks with dragonboat's per-step hand-off: after every tick one rg_get_update
    (slot-0 replicas = one node's share; UPDATE_ALL: hard states + appended entries to persist,
    committed entries to apply, snapshot events, ready reads, all in one staging pass and one D2H)
    and one rg_commit_update(RG_COMMIT_APPLIED), the host reading the sections in place. Host wall time."""
    import ctypes as C
    import torch
    from raftd_amd.engine import Update, UPDATE_ALL, COMMIT_APPLIED
    u = Update()
    nb = ne = 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tick()
        if eng.L.rg_get_update(eng.h, slot_mask, UPDATE_ALL, C.byref(u)) != 0:
            raise RuntimeError(f"rg_get_update: {eng.L.rg_last_error().decode()}")
        ne += u.persist.n_entries + u.committed.n_entries
        nb += u.persist.payload_bytes + u.committed.payload_bytes
        if eng.L.rg_commit_update(eng.h, C.byref(u), COMMIT_APPLIED) != 0:
            raise RuntimeError(f"rg_commit_update: {eng.L.rg_last_error().decode()}")
    el = time.perf_counter() - t0
    return {"value": G * steps / el, "unit": "group-steps/s", "steps": steps, "ms_per_step": el * 1e3 / steps,
            "entry_rows_per_step": ne / steps, "payload_bytes_per_step": nb / steps,
            "note": "tick + rg_get_update(UPDATE_ALL, slot mask 1) + rg_commit_update(RG_COMMIT_APPLIED) per step: "
                    "the single GetUpdate / Commit hand-off (the slot-0 replicas' states, entries to persist as term "
                    "runs + {len, crc} with their Cmds, committed entries as runs + {len, crc} by reference to those "
                    "Cmds (each Cmd crosses PCIe once), snapshots, reads), sections read in place from pinned memory; "
                    "PCIe-bound at full batches"}


def ingest(eng, G, E, P, steps, seed=7):
    """The client ingest path (SURVEY §8b rg_propose ≈ NodeHost.Propose): every step each leader's
    E Cmds of P bytes (host memory, pageable, the way a cgo shim hands Go []byte over) are staged by
    one rg_propose call for all G shards, then the tick runs; host wall time per step, so the
    figure includes the host-side staging and the H2D copy of the Cmd bytes."""
    import ctypes as C
    import numpy as np
    import torch
    from raftd_amd.engine import Proposal
    props = (Proposal * G)()
    a = np.frombuffer(props, dtype=np.dtype([("group", "<u8"), ("slot", "<u4"), ("count", "<u4"), ("first", "<u8")]))
    a["group"] = np.arange(G)
    a["slot"] = 0
    a["count"] = E
    a["first"] = np.arange(G, dtype=np.uint64) * E
    lens = np.full(G * E, P, np.uint32)
    blob = np.random.default_rng(seed).integers(0, 256, G * E * P, dtype=np.uint8)

    def step():
        rc = eng.L.rg_propose(eng.h, props, G, blob.ctypes.data, lens.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"rg_propose: {eng.L.rg_last_error().decode()}")
        eng.tick_device()

    def measure():
        step()  # warm: staging buffers grow once
        torch.cuda.synchronize()
        c0 = eng.sum_committed()
        t0 = time.perf_counter()
        tp = 0.0
        for _ in range(steps):
            a0 = time.perf_counter()
            rc = eng.L.rg_propose(eng.h, props, G, blob.ctypes.data, lens.ctypes.data)
            tp += time.perf_counter() - a0
            if rc != 0:
                raise RuntimeError(f"rg_propose: {eng.L.rg_last_error().decode()}")
            eng.tick_device()
        eng.sync()
        el = time.perf_counter() - t0
        committed = eng.sum_committed() - c0
        nb = G * E * P
        return {"value": G * steps / el, "unit": "group-steps/s", "steps": steps, "ms_per_step": el * 1e3 / steps,
                "propose_ms_per_step": tp * 1e3 / steps, "cmd_bytes_per_step": nb,
                "ingest_GBps": nb * steps / el / 1e9, "propose_GBps": nb * steps / tp / 1e9 if tp else None,
                "commits_per_step": committed / steps}

    out = measure()
    out["note"] = ("per step: one rg_propose of G batches x E Cmds from pageable host memory (validation, staging "
                   "into pinned memory by host threads, H2D copies of the staged pieces overlapping the copying, "
                   "descriptor kernel), then rg_tick_device with no tick-input proposals; host wall time")
    # the same buffer registered (rg_host_register, as a cgo shim would pin its Cmd arena once): the
    # Cmds move by DMA straight out of it
    eng.host_register(blob.ctypes.data, blob.nbytes)
    try:
        reg = measure()
    finally:
        eng.host_unregister(blob.ctypes.data)
    reg["note"] = "the same, with the payload buffer registered once (rg_host_register): DMA straight from it"
    out["registered"] = reg
    return out


def graph_ticks(eng, pt, pc, G, k=10, reps=4):
    """The multi-tick path (rg_tick_device_n, RG_TICKN_GRAPH): the same steady-state ticks, k per
    captured HIP graph, one hipGraphLaunch per k ticks; host wall time per tick."""
    import torch
    eng.tick_device_n(k, pt.data_ptr(), pc.data_ptr())  # capture + first replay
    eng.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.tick_device_n(k, pt.data_ptr(), pc.data_ptr())
    eng.sync()
    el = time.perf_counter() - t0
    out = {"value": G * k * reps / el, "unit": "group-steps/s", "ticks": k * reps, "ticks_per_graph": k,
           "ms_per_step": el * 1e3 / (k * reps),
           "note": "rg_tick_device_n(k, RG_TICKN_GRAPH): k ticks per hipGraphLaunch, parameter blocks written "
                   "into the graph's pinned slots before each launch; host wall time"}
    if eng.cfg["payload_bytes"] == 0 and eng.cfg["replicas"] <= 4:  # the resident control kernel
        kr = 32
        eng.tick_device_n(kr, pt.data_ptr(), pc.data_ptr(), resident=True)
        eng.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.tick_device_n(kr, pt.data_ptr(), pc.data_ptr(), resident=True)
        eng.sync()
        el = time.perf_counter() - t0
        out["resident"] = {"value": G * kr * reps / el, "ms_per_step": el * 1e3 / (kr * reps), "ticks_per_launch": kr,
                           "note": "rg_tick_device_n(k, RG_TICKN_RESIDENT): k ticks in one launch of the resident "
                                   "control kernel (metadata-only engines); host wall time"}
    return out


def pmc_traffic(kernel="bulk_kernel", wire=False, spread=False):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary of the
    same bench mode (profiles/r*_pmc_summary.json; *_wire_* = the --wire-all runs, *_spread_* =
    the spread placement with column halves, profiled as one rank whose messages all cross the
    wire — the launch shape of every rank at N > 1)."""
    def mode(f):
        b = os.path.basename(f)
        if any(t in b for t in ("_c5", "_c2", "_c3", "_c4", "_shape")):
            return "shape"  # another workload's profile (C2-C5 shapes): never the headline's traffic
        return "spread" if "_spread_" in b else "wire" if "_wire_" in b else "plain"
    want = "spread" if spread else "wire" if wire else "plain"
    files = [f for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_summary.json"))) if mode(f) == want]
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    k = d.get("kernels", {}).get(kernel)
    if not k:
        return None, None
    return k.get("hbm_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        sys.exit(2)
    if args.dry_run:
        dry_run(args, rank, world)
        return
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = int(os.environ.get("RAFTD_BENCH_DEVICE", local))
    import torch

    dist = None
    rehearse = world == 1 and args.placement == "spread" and args.wire_all  # N > 1 path on one rank
    if rehearse:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29561")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if world > 1 or rehearse:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.backend)
        world = dist.get_world_size()  # the world the collectives (RCCL with nccl) initialised with
    else:
        torch.cuda.set_device(local)
    from raftd_amd import Engine
    from raftd_amd.cluster import DistEngine

    G, R, E, P = args.groups, args.replicas, args.entries, args.payload
    placement = args.placement or ("spread" if world > 1 else "colocated")
    spread = placement == "spread" and (world > 1 or rehearse)
    stream = torch.cuda.Stream()  # a real (non-null) stream: the engine launches on it, events time it
    torch.cuda.set_stream(stream)
    common = dict(replicas=R, log_capacity=args.log_capacity, payload_bytes=P, max_entries_per_msg=E, device=local)
    wire = None
    if spread:  # one cluster of world x G groups, replicas spread over the GPUs
        wire = DistEngine(groups=G, halves=args.halves, seed=0x5EED, wire_all=1 if rehearse else 0,
                          fixed=None if args.sizing is None else args.sizing == "fixed",
                          exchange=args.exchange, **common)
        host, eng = wire, wire.eng  # host: aggregates over the halves; eng: the first half
        Gt = G * world
    else:  # an independent engine per GPU (its own G groups)
        eng = Engine(groups=G, seed=0x5EED + rank, wire_all=1 if args.wire_all else 0, **common)
        eng.set_stream(stream.cuda_stream)
        if args.wire_all:
            wire = SelfWire(eng, torch)
        host = eng
        Gt = G
    step = wire or eng
    bring_up(host, step.tick, Gt, R)
    pt = torch.zeros(Gt, dtype=torch.uint8, device="cuda")
    pc = torch.full((Gt,), E, dtype=torch.int32, device="cuda")  # read as uint32 by the kernel
    # settle into the steady state before the warm-up steps: until every log ring has wrapped once
    # (L / E ticks: the first pass writes ring slots and stream pages nothing has touched yet, and the
    # first snapshots and compactions come on it). Measured (scripts/timing_probe.py, r05u): the first
    # 20 ticks after bring-up run 1.352 ms each, later ones 1.294-1.300 ms
    settle = min(64, args.log_capacity // max(E, 1) + 8)
    for _ in range(settle):
        step.tick_device(pt.data_ptr(), pc.data_ptr())
    for _ in range(max(args.warmup, 1)):
        step.tick_device(pt.data_ptr(), pc.data_ptr())
    traffic = host.last_tick_traffic()  # counts of a steady-state tick (outside the timed region)
    c0 = host.sum_committed()
    pipelined = spread and args.halves > 1
    if pipelined:
        wire.prime()  # the last warm-up tick's exchange is in flight when the timer starts
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    xev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    def one_step(i):
        """One step; returns the bytes this rank sent to other ranks."""
        if pipelined:  # each half: finish its exchange, tick, start the next exchange
            wire.step_device(pt.data_ptr(), pc.data_ptr())
            return wire.wire_bytes
        sent = 0
        if wire:
            if i is not None:
                xev[i][0].record(stream)
            wire.exchange()
            if i is not None:
                xev[i][1].record(stream)
            sent = wire.wire_bytes
        for e in (wire.parts if spread else [eng]):
            e = e.eng if spread else e
            e.tick_device(pt.data_ptr() + (e.cfg["column_base"] * world if spread else 0),
                          pc.data_ptr() + 4 * (e.cfg["column_base"] * world if spread else 0))
        return sent

    # the roofline kernel, live: HIP events around bulk_kernel on every TIMING_EVERY-th tick of the
    # timed region (each timed event record costs its tick tens of µs on this runtime: timing every
    # tick made the step 8% slower, r03d)
    if spread:  # the halves' bulk launches on one timeline: their span per tick (DistEngine.kernel_span_ms)
        from raftd_amd.engine import timing_epoch
        timing_epoch(local)
    host.timing(True, bulk_only=True, every=TIMING_EVERY)
    wire_bytes = 0
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        wire_bytes += one_step(i)
    if pipelined:
        wire.drain()  # the last step's exchanges complete inside the timed region
    host.join()  # the stream waits for the last tick's payload stage before the end event
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    dev_ms = ev0.elapsed_time(ev1)
    kms = host.kernel_ms()
    span = host.kernel_span_ms("bulk") if spread else None
    c1 = host.sum_committed()  # before the control-timing steps below
    # the state the timed ticks left (before the extra phases below run more ticks): invariant bits,
    # drops, the hand-off count, the page pool (a shape whose log outgrows the pool without compaction
    # — C5's 1 entry per leader per tick at SnapshotEntries 1000 — must show it here, not in the timed ticks)
    va = eng.replica_array()  # every replica of this rank's first engine
    ctl_slow = None
    fn = getattr(eng.L, "rg_debug_ctl_slow", None)
    if fn is not None:  # replicas of the last tick whose step left the control fast path
        import ctypes as C
        fn.argtypes, fn.restype = [C.c_void_p, C.POINTER(C.c_uint32)], C.c_int
        n_slow = C.c_uint32()
        if fn(eng.h, C.byref(n_slow)) == 0:
            ctl_slow = n_slow.value
    errs, drops = int((va["err"] != 0).sum()), int(va["drops"].sum())
    pool_timed = eng.pool_stats() if P else None
    del va
    # control_kernel duration from a few more steps after the timed region (timing both kernels
    # adds two event records per tick, which the timed region does without)
    host.timing(True)
    for _ in range(CONTROL_TIMING_STEPS):
        one_step(None)
    if pipelined:
        wire.drain()
    kms["control"] = host.kernel_ms()["control"]
    host.timing(False)
    # the same steps once more with no timing events at all (the roofline's bulk events are two
    # event records per tick in the timed region): what the event records themselves cost
    torch.cuda.synchronize()
    u0 = time.perf_counter()
    for _ in range(args.steps):
        one_step(None)
    if pipelined:
        wire.drain()
    host.join()
    torch.cuda.synchronize()
    untimed_ms = (time.perf_counter() - u0) * 1e3 / args.steps
    # a shape whose appends outgrow the page pool without compaction (C5's one entry per leader per tick at
    # SnapshotEntries 1000) ran the repeat on an exhausted pool: not a comparable step, so not reported
    untimed_note = None
    if P and eng.pool_stats()["failed"]:
        untimed_ms = None
        untimed_note = "not measured: the page pool ran dry after the timed ticks (see pool_after_timed_ticks)"
    graph = graph_ticks(eng, pt, pc, G) if not spread and not args.wire_all else None
    x_ms = sum(a.elapsed_time(b) for a, b in xev) / args.steps if wire and not pipelined else 0.0
    e2e = None
    if not spread:
        e2e = copyback_schedules(eng, lambda: one_step(None), G, steps=max(4, min(args.steps, 12)))
        hand_off(eng, lambda: one_step(None), G, steps=2)  # warm: the pinned update buffer grows here
        e2e["hand_off"] = hand_off(eng, lambda: one_step(None), G, steps=max(3, min(args.steps, 8)))
    apply = apply_copyback(eng, torch)
    ing = ingest(eng, G, E, P, steps=max(3, min(args.steps, 8))) if args.ingest and not spread and P else None
    copy_gbs = hbm_copy_ceiling(eng)
    t = torch.tensor([wall, dev_ms, float(c1 - c0), x_ms, float(wire_bytes)], dtype=torch.float64,
                     device="cuda" if args.backend == "nccl" else "cpu")
    if dist:
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        wall, dev_max, commits = tmax[0].item(), tmax[1].item(), tsum[2].item()
        x_ms, wire_max = tmax[3].item(), tmax[4].item()
    else:
        dev_max, commits, wire_max = dev_ms, float(c1 - c0), float(wire_bytes)
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    K = args.steps
    group_steps = world * G * K / wall
    transport = exchange_transport(spread, bool(args.wire_all), args.exchange, args.backend if dist else "none",
                                   bool(wire.fixed) if spread else True)
    if spread:
        par = (f"{world * G} groups; replica slot s of group g on GPU (g mod {world} + off(s, g div {world})) mod "
               f"{world}, every replica of a group on its own GPU, followers spread evenly over the peers; "
               f"cross-GPU messages once per tick by {transport}"
               + (f" and column half ({args.halves} halves per GPU, exchange pipelined behind the other half's tick)"
                  if args.halves > 1 else "")
               + (" [rehearsal: one rank, every message through the wire to itself]" if rehearse else ""))
    elif args.wire_all:
        par = "1 GPU, every message through the wire pack/unpack path to itself (measurement)"
    else:
        par = f"groups sharded over {world} GPU(s), replicas co-located (no exchange)"
    bulk_ms = kms["bulk"][0] / max(kms["bulk"][1], 1)
    bulk_sum_ms = bulk_ms
    if span and span[1]:  # column halves: the span of their launches per tick, not the sum of the durations
        bulk_ms = span[0] / span[1]
    ctl_ms = kms["control"][0] / max(kms["control"][1], 1)
    # metadata-only (P = 0): no payload stage is launched, the control kernel is the tick
    meta_only = kms["bulk"][1] == 0
    rk_ms = ctl_ms if meta_only else bulk_ms
    rk_bytes = traffic["algorithmic_bytes"] if meta_only else traffic["bulk_bytes"]
    achieved = rk_bytes / (rk_ms / 1e3) / 1e9 if rk_ms > 0 else 0.0
    # PMC bytes come from a committed profile of the same mode and launch size; the N > 1 spread
    # engines (column halves, wire jobs) have none, so their traffic is left unmeasured
    hbm, src = pmc_traffic(wire=bool(args.wire_all), spread=spread)
    if (G, R, E, P, args.log_capacity) != (65536, 3, 64, 256, 2048):  # the profiles are of this workload
        hbm, src = None, "no PMC profile of this workload"
    if spread and hbm is not None:  # the spread profile is per half (bench default --halves 2); here per tick
        hbm = hbm * 2 if args.halves == 2 else None
    out = {
        "metric": METRIC,
        "value": group_steps,
        "unit": "group-steps/s",
        "n_gpus": world,
        "backend": args.backend if dist else None,
        "ranks_share_one_gpu": bool(dist) and world > 1 and "RAFTD_BENCH_DEVICE" in os.environ,
        "steps": K,
        "warmup": args.warmup,
        "settle_ticks": settle,  # steady-state ticks after bring-up, before the warm-up steps
        "ms_per_step": wall * 1e3 / K,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic",
        "config": {
            "workload": f"{G} groups x {R} replicas per GPU, steady-state leaders, {E}-entry batches of "
                        f"{P}-B payloads + CRC32 per tick, raftd Raft config (ElectionRTT 10, HeartbeatRTT 1, "
                        f"CheckQuorum, SnapshotEntries 1000, CompactionOverhead 5)",
            "groups_per_gpu": G, "replicas": R, "entries_per_batch": E, "payload_bytes": P,
            "log_capacity": args.log_capacity, "placement": "spread" if spread else placement,
            "parallelism": par,
        },
        "commits_per_sec": commits / wall,
        "replica_steps_per_sec": group_steps * R,
        "device_ms_per_step": dev_max / K,
        "ms_per_step_without_timing_events": untimed_ms,
        "ms_per_step_without_timing_events_note": untimed_note,
        "replicas_with_invariant_errors": errs,
        "pool_after_timed_ticks": pool_timed,
        "drops_total": drops,
        "drops_note": "messages / batches the engine dropped by its own bounded-buffer rules (K_MAX per pair per "
                      "tick, ring capacity, forward hop limit) since bootstrap, summed over this rank's replicas",
        "commits_expected_per_step": world * G * E,
        "commits_measured_per_step": commits / K,
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": hbm,
            "traffic_source": src,
            "kernel": "rg::control_kernel" if meta_only else "rg::bulk_kernel",
            "box_copy_ceiling_GBps": copy_gbs,
            "frac_of_box_copy_ceiling": achieved / copy_gbs if copy_gbs else None,
            "kernel_ms": rk_ms,
            "launches_timed": kms["bulk"][1],
            "launches_timed_note": f"HIP events around bulk_kernel on every {TIMING_EVERY}th tick of the timed region",
            "per": ("tick: wall-clock time the column halves' bulk_kernel launches of a tick ran (the union of "
                    "their intervals on one timeline, rg_timing_epoch)") if spread and args.halves > 1 else "launch",
            "bulk_ms_summed_over_halves": bulk_sum_ms if spread and args.halves > 1 else None,
            "algorithmic_bytes_per_launch": rk_bytes,
            "tick_algorithmic_bytes": traffic["algorithmic_bytes"],
            "tick_counts": {k: v for k, v in traffic.items() if k not in ("algorithmic_bytes", "bulk_bytes")},
        },
        "kernels_ms": {"control_kernel": ctl_ms, "bulk_kernel": bulk_ms},
        "control_fast_path": {"enabled": True,
                              "slow_replicas_last_tick": ctl_slow,
                              "note": "control_kernel time = control_fast_kernel (the steady-state branches, compiled per "
                                      "role: three waves per SIMD at R <= 3) + control_slow_kernel (the full step for the "
                                      "replicas the fast kernel handed off); engines of <= 64K replicas run "
                                      "control_fastfb_kernel instead (the full step inside the same launch)"},
        "exchange": None if not wire else {
            "mode": (f"pipelined over {args.halves} column halves: one half's all-to-all overlaps the other's "
                     "unpack + tick + pack" if pipelined else "serial: plan + pack + all-to-all + unpack, then tick"),
            "ms_per_step": x_ms if not pipelined else None,
            "transport": transport,
            "bytes_sent_per_step_max_rank": wire_max / K,
            "bound_ms": xgmi_bound_ms(wire_max / K, world),
            "bound_note": "the busiest rank's outbound bytes per step / ((N - 1) xGMI links x "
                          f"{XGMI_LINK_GBS:.0f} GB/s), traffic spread evenly over the peers (DESIGN.md §6); "
                          "a step at N > 1 cannot be shorter. None at N = 1",
            "achieved_GBps_per_rank": ((wire_max / K) / (x_ms / 1e3) / 1e9 if x_ms > 0 else
                                       (wire_max / K) / (wall / K) / 1e9),
            "xgmi_peak_GBps_per_rank": min(max(world - 1, 1), 7) * XGMI_LINK_GBS,
            "xgmi_frac": (((wire_max / K) / (x_ms / 1e3) / 1e9 if x_ms > 0 else (wire_max / K) / (wall / K) / 1e9)
                          / (min(max(world - 1, 1), 7) * XGMI_LINK_GBS)),
            "note": "bytes = the regions this rank sends to other ranks per step; serial mode times the exchange "
                    "with events on the bench stream, pipelined mode reports bytes / step time (a lower bound)",
        },
        "device_bytes": host.device_bytes,
        "apply_copyback": apply,
        "e2e_with_apply": e2e,
        "graph": graph,
    }
    if ing:
        out["ingest"] = ing
    if not args.no_cpu_baseline and world == 1:  # rank 0 at N=1 only
        out["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
