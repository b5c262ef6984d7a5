#!/bin/bash
# r06 final build, call B: the rocprofv3 passes (kernel trace + FETCH / WRITE) of the headline and C5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/profile.sh r06_final --steps 10 --warmup 3 --no-cpu-baseline || exit 1
bash scripts/profile.sh r06_final_c5 --groups 1048576 --entries 1 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
