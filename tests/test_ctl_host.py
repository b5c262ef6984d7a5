"""The engine's control step (raftgpu_control.h, i.e. control_kernel<R>'s body) compiled for the
CPU by tests/native/ctl_host.cpp, checked tick by tick against the C oracle: replica state,
every message (header + inline entry terms) and every log entry's term/type. Payload bytes and
CRCs belong to the bulk kernel and are covered by the GPU tests. One case runs under
AddressSanitizer + UBSan in a subprocess."""
import os
import subprocess
import sys

import numpy as np
import pytest

import kat_scenarios as K
from engines import make

HERE = os.path.dirname(os.path.abspath(__file__))


def inputs(rng, G, R, emax):
    pt = rng.integers(0, R, G).astype(np.uint8)
    pt[rng.random(G) < 0.3] = 0xFF
    pc = rng.integers(1, emax + 1, G).astype(np.uint32)
    camp = (rng.random(G * R) < 0.02).astype(np.uint8)
    iso = (rng.random(G * R) < 0.05).astype(np.uint8)
    return pt, pc, camp, iso


def xcheck(kind, seed, G, R, T, p_cc=0.0, wire_all=0, p_read=0.0, **cfg):
    """p_cc: per group and tick, the probability of a membership change. wire_all: the
    control step reads every message from the remote inbox planes (the harness emulates the wire).
    p_read: per replica and tick, the probability of a ReadIndex request (the ready reads must match)."""
    kw = dict(groups=G, replicas=R, payload_bytes=16, max_entries_per_msg=8, log_capacity=64,
              snapshot_entries=20, compaction_overhead=5, drop_ppm=150000, seed=seed)
    kw.update(cfg)
    a, b = make(kind, wire_all=wire_all, **kw), make("c", **kw)
    a.bootstrap()
    b.bootstrap()
    rng = np.random.default_rng(seed)
    for t in range(T):
        if p_cc:
            from test_oracle import random_ccs
            for c in random_ccs(rng, G, R, p_cc):
                assert b.config_change(*c) == 0 and a.config_change(*c) == 0
        if p_read:
            from test_oracle import random_reads
            reqs = random_reads(rng, G, R, t, p=p_read)
            a.read_index(reqs)
            b.read_index(reqs)
        ins = inputs(rng, G, R, kw["max_entries_per_msg"])
        a.tick(*ins)
        b.tick(*ins)
        for rid in range(G * R):
            vb = b.replica(rid)
            assert a.replica(rid) == vb, (seed, t, rid)
            # the step's hand-off word (apply window, snapshot events) decodes to the oracle's
            f, (kind, restored, _, _) = a.feed(rid), b.snapshot_event(rid)
            assert (f["apply_lo"], f["restored"], f["took"]) == (b.apply_lo(rid), restored, bool(kind & 1)), \
                (seed, t, rid, f)
            if f["persist_lo"] != 2 ** 64 - 1:  # entries written: the word marks the persist bit too
                assert f["persist"] and f["persist_lo"] <= vb["last"], (seed, t, rid, f)
            if p_read:
                assert a.read_ready(rid) == b.read_ready(rid), (seed, t, rid)
            for d in range(R):
                assert a.msgs(rid, d) == b.msgs(rid, d), (seed, t, rid, d)
            for i in range(vb["marker"] + 1, vb["last"] + 1):
                eb = b.entry(rid, i)
                assert a.entry(rid, i) == dict(term=eb["term"], type=eb["type"]), (seed, t, rid, i)


@pytest.mark.parametrize("R", [1, 2, 3, 4, 5, 7, 8])
def test_control_step_matches_oracle(R):
    xcheck("ctl", 10 + R, G=5, R=R, T=120)


@pytest.mark.parametrize("R,wire", [(3, 0), (5, 0), (8, 0), (3, 1), (5, 1)])
def test_slim_full_step_matches_oracle(R, wire):
    """The SLIM build of the full step (control_slow_kernel / control_kernel: narrower load batches)
    under chaos, membership changes and reads, local and remote inboxes."""
    xcheck("ctl-slim", 110 + R, G=5, R=R, T=120, wire_all=wire, p_cc=0.03 if R > 2 else 0.0, p_read=0.2)


@pytest.mark.parametrize("R", [2, 3, 5, 8])
@pytest.mark.parametrize("kind", ["ctl", "ctl-fast"])
def test_control_step_over_the_wire_matches_oracle(kind, R):
    """Every plane remote (wire_all; the harness emulates pack + unpack): the step's remote-inbox
    paths — rhdr / rmt / rcnt, uniform WIRE appends on the fast path, records offsets, forwarded
    Proposes with their length words — equal the oracle, with and without the fast path."""
    xcheck(kind, 50 + R, G=5, R=R, T=120, wire_all=1, p_cc=0.03 if R > 2 else 0.0)


@pytest.mark.parametrize("R", [1, 2, 3, 5, 8])
def test_fast_path_matches_oracle(R):
    """The fast-path step (Ctl<R, true>: the steady-state branches, handing every other step to the
    full Ctl<R>) under chaos — loss, isolation, elections, truncation, snapshots — equals the oracle."""
    xcheck("ctl-fast", 30 + R, G=5, R=R, T=120)


@pytest.mark.parametrize("R", [1, 3, 5])
def test_fast_path_latency_build_matches_oracle(R):
    """The small-engine latency build of the fast step (Ctl<R, true, role, LAT = true>: every field
    loaded up front; control_fastfb_kernel and the resident kernel) against the oracle."""
    xcheck("ctl-fastlat", 50 + R, G=5, R=R, T=120)


def test_fast_path_membership_and_heavy_loss():
    xcheck("ctl-fast", 88, G=6, R=5, T=160, drop_ppm=300000, max_msgs_per_pair=4, p_cc=0.05)


@pytest.mark.parametrize("R,P,wire", [(3, 256, 0), (5, 64, 0), (3, 0, 0), (3, 256, 1), (5, 64, 1)])
def test_fast_path_covers_the_steady_state(R, P, wire):
    """Steady-state leaders with a full batch every tick (the benchmark's workload, snapshots and
    compaction included): after the election no replica's step leaves the fast path — with every
    message over the wire too (wire: the multi-GPU step's inbox)."""
    G, E = 8, 16
    kw = dict(groups=G, replicas=R, payload_bytes=P, max_entries_per_msg=E, log_capacity=256,
              snapshot_entries=100, compaction_overhead=5, seed=9)
    a, b = make("ctl-fast", wire_all=wire, **kw), make("c", **kw)
    for e in (a, b):
        e.bootstrap()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    pt, pc = np.zeros(G, np.uint8), np.full(G, E, np.uint32)
    for t in range(60):
        ins = dict(campaign=camp) if t == 1 else dict(prop_target=pt, prop_count=pc) if t >= 6 else {}
        if t == 10:
            slow0 = a.slow_lanes
        a.tick(**ins)
        b.tick(**ins)
        for rid in range(G * R):
            assert a.replica(rid) == b.replica(rid), (t, rid)
    assert b.replica(0)["snap_index"] > 0  # the run went through snapshots and compaction
    assert a.slow_lanes == slow0, a.slow_lanes - slow0


@pytest.mark.parametrize("R,wire", [(1, 0), (3, 0), (5, 0), (3, 1), (5, 1)])
@pytest.mark.parametrize("kind", ["ctl", "ctl-fast"])
def test_control_step_read_index_queue(kind, R, wire):
    """ReadIndex under chaos with up to RG_READ_QUEUE requests pending per leader (dragonboat's
    readIndex queue): every state, message and ready read equals the oracle, local and remote inboxes."""
    xcheck(kind, 70 + R, G=5, R=R, T=120, wire_all=wire, p_read=0.35, heartbeat_rtt=2)


def test_control_step_heavy_loss():
    xcheck("ctl", 77, G=6, R=5, T=200, drop_ppm=300000, max_msgs_per_pair=4)


@pytest.mark.parametrize("R,im", [(3, 0), (5, 0b01011), (8, 0), (2, 0b01), (7, 0b1110111)])
def test_control_step_membership_matches_oracle(R, im):
    """ConfigChange proposals through the kernel's step: members, quorum, elections, snapshots."""
    xcheck("ctl", 200 + R, G=5, R=R, T=160, p_cc=0.06, initial_members=im)


@pytest.mark.parametrize("name,fn", [
    ("voter", lambda k: [K.run_voter(k, c) == c["reject"] for c in K.load("kat_voter.json")["cases"]]),
    ("msgapp", lambda k: [K.run_check_msgapp(k, K.load("kat_check_msgapp.json"), c) ==
                          dict(reject=c["reject"], resp_index=c["resp_index"], hint=c["hint"])
                          for c in K.load("kat_check_msgapp.json")["cases"]]),
    ("append", lambda k: [K.run_append(k, K.load("kat_append.json"), c) == c["want"]
                          for c in K.load("kat_append.json")["cases"]]),
    ("ctc", lambda k: [K.run_current_term_commit(k, K.load("kat_current_term_commit.json")) ==
                       [a["want_commit"] for a in K.load("kat_current_term_commit.json")["acks"]]]),
])
def test_control_step_kats(name, fn):
    assert all(fn("ctl"))


@pytest.mark.parametrize("name", sorted(K.PAPER_KATS))
def test_control_step_paper_kats(name):
    assert all(K.PAPER_KATS[name]("ctl"))


def test_control_step_under_asan():
    from native import ctl_host
    ctl_host.build(asan=True)
    pre = ":".join(subprocess.check_output(["gcc", f"-print-file-name={lib}"], text=True).strip()
                   for lib in ("libasan.so", "libubsan.so"))
    code = ("import sys; sys.path[:0] = [%r, %r]; import test_ctl_host as t; "
            "t.xcheck('ctl-asan', 5, G=3, R=3, T=60); t.xcheck('ctl-asan', 6, G=2, R=5, T=60); "
            "t.xcheck('ctl-asan', 7, G=3, R=8, T=80, p_cc=0.08); "
            "t.xcheck('ctl-fast-asan', 8, G=3, R=3, T=80, p_cc=0.05); t.xcheck('ctl-fast-asan', 9, G=2, R=5, T=60); "
            "t.xcheck('ctl-asan', 11, G=3, R=5, T=60, wire_all=1, p_cc=0.05); "
            "t.xcheck('ctl-fast-asan', 12, G=3, R=5, T=60, wire_all=1); t.xcheck('ctl-fast-asan', 13, G=2, R=8, T=60, wire_all=1); "
            "t.xcheck('ctl-slim-asan', 14, G=3, R=5, T=60, p_cc=0.05, p_read=0.2); "
            "import kat_scenarios as K; fx = K.load('kat_check_msgapp.json'); "
            "[K.run_check_msgapp('ctl-asan', fx, c) for c in fx['cases']]; print('ASAN-CLEAN')"
            % (HERE, os.path.dirname(HERE)))
    env = dict(os.environ, LD_PRELOAD=pre, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "ASAN-CLEAN" in r.stdout, r.stderr[-3000:]


def test_control_step_c3_shape():
    """C3's per-rank shape (8,192 columns x 5, L 512, 64-entry batches of 256 B, SnapshotEntries
    200) for 24 ticks, past a ring wrap and snapshots, against the oracle on sampled replicas: the
    index arithmetic at the size where the GPU fault appeared."""
    G, R = 8192, 5
    cfg = dict(groups=G, replicas=R, log_capacity=512, payload_bytes=256, max_entries_per_msg=64,
               snapshot_entries=200, seed=0xC3)
    a, b = make("ctl", **cfg), make("c", **cfg)
    a.bootstrap()
    b.bootstrap()
    camp = np.zeros(G * R, np.uint8)
    camp[0::R] = 1
    pt, pc = np.zeros(G, np.uint8), np.full(G, 64, np.uint32)
    for t in range(24):
        ins = dict(campaign=camp) if t == 1 else (dict(prop_target=pt, prop_count=pc) if t >= 6 else {})
        a.tick(**ins)
        b.tick(threads=8, **ins)
        if t % 4 == 3:
            for rid in range(0, G * R, 997):
                assert a.replica(rid) == b.replica(rid), (t, rid)
    assert b.replica(0)["committed"] > 512 and b.replica(0)["marker"] > 0


def test_control_step_term_limit():
    """The 36-bit term boundary on the control step compiled for the CPU, as on the oracles."""
    assert K.run_term_limit("ctl", K.TERM_MAX - 1) == ("candidate", K.TERM_MAX, 0, 2)
    assert K.run_term_limit("ctl", K.TERM_MAX) == ("follower", K.TERM_MAX, K.ERR_TERM_LIMIT, 0)


def test_control_step_under_msan():
    """The control step compiled for the CPU under MemorySanitizer (clang's; tests/native/ctl_msan.cpp,
    a stand-alone driver: MSan needs an instrumented executable): no branch, address or store of the
    step depends on a value it never initialised — over the steady C3 shape and chaos, every R, the
    full / fast / latency builds, local and remote inboxes (the control-kernel fault)."""
    clang = "/opt/rocm/lib/llvm/bin/clang++"
    if not os.path.exists(clang):
        pytest.skip("no clang with MemorySanitizer")
    out = os.path.join(HERE, "native", "build", "ctl_msan")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    root = os.path.dirname(HERE)
    deps = [os.path.join(HERE, "native", f) for f in ("ctl_msan.cpp", "ctl_host.cpp")] + \
        [os.path.join(root, "raftd_amd", "csrc", f) for f in ("raftgpu_control.h", "raftgpu_internal.h")] + \
        [os.path.join(root, "include", "raftgpu.h")]
    if not os.path.exists(out) or any(os.path.getmtime(d) > os.path.getmtime(out) for d in deps):
        subprocess.run([clang, "-fsanitize=memory", "-fsanitize-memory-track-origins=2", "-fno-omit-frame-pointer",
                        "-O1", "-g", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                        os.path.join(HERE, "native", "ctl_msan.cpp"), "-o", out], check=True, timeout=900)
    r = subprocess.run([out], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "MSAN-CLEAN" in r.stdout, r.stderr[-3000:]
    probe = subprocess.run([out], capture_output=True, text=True, timeout=600, env=dict(os.environ, CTL_MSAN_PROBE="1"))
    assert probe.returncode != 0 and "use-of-uninitialized-value" in probe.stderr  # the sanitizer is live
