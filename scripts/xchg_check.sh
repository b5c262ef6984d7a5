#!/bin/bash
# rg_wire_exchange on the GPU box: its tests, then the one-rank rehearsal bench (every message
# through the wire, the N > 1 code path) with the Python exchange and with the C-ABI exchange.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_abi.py tests/test_gpu_cluster.py -k "exchange or harness" > gpurun_out/xchg_tests.log 2>&1 || { tail -40 gpurun_out/xchg_tests.log; exit 1; }
tail -3 gpurun_out/xchg_tests.log
for x in torch c; do
  timeout -k 10 300 python bench.py --placement spread --wire-all --no-cpu-baseline --steps 10 --warmup 3 --exchange $x \
    > gpurun_out/rehearse_$x.log 2>&1 || { tail -20 gpurun_out/rehearse_$x.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/rehearse_$x.log').read().strip().splitlines()[-1])
print('$x', round(d['ms_per_step'],3), 'ms/step', d['kernels_ms'], d['exchange']['transport'])"
done
