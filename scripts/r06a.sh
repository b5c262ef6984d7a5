#!/bin/bash
# r06a: in-place replica state. Smoke, the parity subset, the GPU suite, the headline bench, then the
# C5 shape (1M x 3, one entry per leader per tick) and the 64K x 3 headline under rocprofv3 (kernel
# trace, FETCH_SIZE, WRITE_SIZE passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS="smoke parity tests bench" bash scripts/gpu_round.sh || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --groups 1048576 --entries 1 --steps 10 --warmup 3 > gpurun_out/r06a_c5.log 2>&1 || { tail -5 gpurun_out/r06a_c5.log; exit 1; }
tail -1 gpurun_out/r06a_c5.log | cut -c1-600
bash scripts/profile.sh r06a_c5 --groups 1048576 --entries 1 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
bash scripts/profile.sh r06a || exit 1
