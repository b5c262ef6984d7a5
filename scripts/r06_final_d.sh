#!/bin/bash
# r06 final build, call D: the randomised parity soak (5 minutes) and the 2-rank gloo rehearsal of the
# N > 1 launcher, on the build with the speculated parameter chunks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 420 python -u scripts/soak.py 300 7000 > gpurun_out/r06_final_soak.log 2>&1 || { tail -20 gpurun_out/r06_final_soak.log; exit 1; }
tail -3 gpurun_out/r06_final_soak.log
STEPS="rehearse" bash scripts/gpu_round.sh || exit 1
