#!/bin/bash
# smoke + GPU tests + bench on the GPU box; stops at the first failure or runtime fault.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fault() { grep -q "HSA_STATUS_ERROR\|illegal memory access\|Memory access fault" "$1"; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ] || fault gpurun_out/smoke.log; then echo "SMOKE FAILED rc=$rc"; exit 1; fi
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -25 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] || fault gpurun_out/gpu_tests.log; then echo "GPU TESTS FAILED rc=$rc"; exit 1; fi
if [ "${1:-}" = "bench" ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.log 2>&1; rc=$?
  tail -2 gpurun_out/bench.log
  if [ $rc -ne 0 ] || fault gpurun_out/bench.log; then echo "BENCH FAILED rc=$rc"; exit 1; fi
fi
echo ALL-OK
