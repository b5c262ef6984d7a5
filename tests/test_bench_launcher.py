"""bench.py --gpus N started as one process launches N ranks. CPU only: --dry-run
ranks join a gloo group and report the world size they agree on, without touching a GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=180, env=e)


def test_gpus_two_spawns_two_ranks():
    r = _run(["--gpus", "2", "--backend", "gloo", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["ranks_agreeing"] == 2 and line["dry_run"]


def test_gpus_four_spawns_four_ranks():
    r = _run(["--gpus", "4", "--backend", "gloo", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 4


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "2", "--dry-run"], env={"WORLD_SIZE": "3", "RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE 3" in r.stderr


def test_transport_label_names_the_exchange_that_ran():
    """the N > 1 line's `parallelism` label and exchange.transport come from one function
    of --exchange / backend / sizing, so the label cannot name a transport the step did not use."""
    sys.path.insert(0, ROOT)
    import bench
    t = bench.exchange_transport(True, False, "torch", "nccl", True)
    assert "batch_isend_irecv" in t and "rg_wire_exchange" not in t and "fixed-capacity" in t
    c = bench.exchange_transport(True, False, "c", "nccl", True)
    assert "rg_wire_exchange" in c and "ncclSend" in c and "batch_isend_irecv" not in c
    assert "gloo" in bench.exchange_transport(True, False, "c", "gloo", False)
    assert "exactly sized" in bench.exchange_transport(True, False, "torch", "nccl", False)
    assert "gloo" in bench.exchange_transport(True, False, "torch", "gloo", True)
    assert bench.exchange_transport(False, True, "torch", "nccl", True) == "device copy (one engine)"
    assert bench.exchange_transport(False, False, "torch", "nccl", True) is None


def test_xgmi_bound():
    """exchange.bound_ms: the busiest rank's bytes over its N - 1 links at XGMI_LINK_GBS each."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.xgmi_bound_ms(1.34e9, 1) is None
    assert abs(bench.xgmi_bound_ms(1.34e9, 2) - 1.34e9 / 153e9 * 1e3) < 1e-9
    assert abs(bench.xgmi_bound_ms(2.1e9, 8) - 2.1e9 / (7 * 153e9) * 1e3) < 1e-9


def test_kernel_span_is_the_union_of_the_halves_intervals():
    """The N > 1 line's bulk time per tick: overlapping halves (their own streams) count their overlap
    once; halves on one stream with other work between them count only the launches."""
    sys.path.insert(0, ROOT)
    import numpy as np
    from raftd_amd.cluster import DistEngine

    class E:
        def __init__(self, ev):
            self.ev = ev

        def kernel_events(self, kernel):
            t, a, b = zip(*self.ev)
            return np.array(t, np.uint64), np.array(a), np.array(b)

    class P:
        def __init__(self, ev):
            self.eng = E(ev)

    d = DistEngine.__new__(DistEngine)
    d.parts = [P([(4, 0.0, 1.0), (8, 10.0, 11.0)]), P([(4, 0.5, 1.5), (8, 12.0, 13.0)])]
    tot, n = d.kernel_span_ms()
    assert n == 2 and abs(tot - (1.5 + 2.0)) < 1e-12
