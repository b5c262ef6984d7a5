"""The committed trace fixtures (tests/golden/trace_r*_chaos.json) replayed on the HIP engine —
one engine, and the same shard set spread over two ranks — against the fixtures' per-tick
digests of every replica view and outbound message and their final views: recorded traces give
bit-identical results on the GPU without consulting the oracle at run time."""
import hashlib
import json

import numpy as np
import pytest

import kat_scenarios as K
from engines import make
from test_gpu_parity import random_inputs

pytestmark = pytest.mark.gpu


def digest(e, G, R):
    h = hashlib.sha256()
    views = e.replicas()
    for rid in range(G * R):
        h.update(json.dumps(views[rid], sort_keys=True).encode())
        for d in range(R):
            h.update(json.dumps(e.msgs(rid, d), sort_keys=True).encode())
    return h.hexdigest()[:16], views


@pytest.mark.parametrize("name,ranks", [("trace_r3_chaos.json", 1), ("trace_r3_chaos.json", 2),
                                        ("trace_r3_chaos.json", 4), ("trace_r5_chaos.json", 1),
                                        ("trace_r5_chaos.json", 3)])
def test_trace_fixture_on_gpu(name, ranks):
    fx = K.load(name)
    cfg = fx["config"]
    if ranks == 1:
        e = make("gpu", **cfg)
    else:
        from raftd_amd.cluster import LoopbackCluster
        e = LoopbackCluster(ranks=ranks, **cfg)
    e.bootstrap()
    G, R = cfg["groups"], cfg["replicas"]
    rng = np.random.default_rng(fx["input_seed"])
    views = None
    for t in range(fx["ticks"]):
        e.tick(*random_inputs(rng, G, R, cfg["max_entries_per_msg"]))
        d, views = digest(e, G, R)
        assert d == fx["digests"][t], f"tick {t}"
    assert views == fx["final"]
