#!/bin/bash
# r06 final build, call A: smoke, the GPU suite, the default bench line (the driver's command), the
# randomised parity soak (5 minutes), and the 2-rank gloo rehearsal of the N > 1 launcher.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BENCH_ARGS=" " STEPS="smoke tests bench" bash scripts/gpu_round.sh || exit 1
timeout -k 10 420 python -u scripts/soak.py 300 6000 > gpurun_out/r06_final_soak.log 2>&1 || { tail -20 gpurun_out/r06_final_soak.log; exit 1; }
tail -3 gpurun_out/r06_final_soak.log
STEPS="rehearse" bash scripts/gpu_round.sh || exit 1
