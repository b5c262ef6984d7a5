#!/bin/bash
# A/B of an environment switch on one box: bench.py with each setting, alternated.
# usage: VAR=RAFTGPU_CTL_FAST VALS="1 0" bash scripts/ab_env.sh [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in $VALS; do
    tag=${VAR}_${v}_$rep
    timeout -k 10 ${AB_TIMEOUT:-200} env $VAR=$v python bench.py --no-cpu-baseline "$@" > gpurun_out/abenv_$tag.log 2>&1 || { tail -5 gpurun_out/abenv_$tag.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/abenv_$tag.log').read().strip().splitlines()[-1])
print('$tag', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, d.get('control_fast_path',{}).get('slow_replicas_last_tick'))"
  done
done
