"""One scenario interface over the three step implementations.

kind "c"   — oracle/oracle.c via oracle/pyoracle.py (the parity oracle)
kind "py"  — oracle/pyraft.py (independent restatement, cross-check only)
kind "gpu" — the HIP engine through the C-ABI (raftd_amd.engine.Engine); needs a GPU

All expose: bootstrap(), tick(prop_target, prop_count, campaign, isolate, flags),
replica(rid) -> dict, msgs(rid, dst) -> list[dict], entry(rid, index) -> dict|None,
import_replica(rid, view, terms, types=None, payloads=None), deliver(rid_src, **fields).
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from oracle import pyoracle, pyraft  # noqa: E402

KINDS_CPU = ("c", "py")


def make(kind: str, **cfg):
    if kind == "c":
        return pyoracle.Oracle(**cfg)
    if kind == "py":
        return pyraft.Sim(**cfg)
    if kind == "gpu":
        from raftd_amd.engine import Engine
        return Engine(**cfg)
    if kind in ("ctl", "ctl-asan", "ctl-fast", "ctl-fast-asan", "ctl-fastlat", "ctl-fastlat-asan", "ctl-slim",
                "ctl-slim-asan"):
        from native.ctl_host import CtlHost
        fast = 3 if "slim" in kind else 2 if "fastlat" in kind else 1 if "fast" in kind else 0
        return CtlHost(asan=kind.endswith("asan"), fast=fast, **cfg)
    raise ValueError(kind)


def view(R: int, **kw) -> dict:
    """A replica view with defaults; remote arrays padded to 8."""
    v = dict(term=1, vote=0, leader=0, committed=0, applied=0, last=0, marker=0, marker_term=0,
             snap_index=0, snap_term=0, cap_base=0, role=0, election_tick=0, heartbeat_tick=0,
             rand_timeout=10, rng_ctr=1, granted=0, responded=0, active=0, err=0, drops=0)
    v.update(kw)
    for f in ("match", "next", "rsnap", "rstate"):
        x = list(v.get(f, [0] * R))
        v[f] = x + [0] * (8 - len(x))
    return v


def log_terms(e, rid):
    r = e.replica(rid)
    return [e.entry(rid, i)["term"] for i in range(r["marker"] + 1, r["last"] + 1)]


def leader_view(R: int, slot: int, term: int, log: list, committed: int = 0, **kw) -> dict:
    """Leader right after becomeLeader+appendEntries: remotes next = last_before_noop+1."""
    last = len(log)
    nxt = [last for _ in range(R)]  # last-before-no-op + 1 == len(log) when log ends with no-op
    match = [0] * R
    match[slot] = last
    nxt[slot] = last + 1
    return view(R, term=term, vote=slot + 1, leader=slot + 1, role=2, last=last, committed=committed,
                applied=committed, match=match, next=nxt, **kw)
