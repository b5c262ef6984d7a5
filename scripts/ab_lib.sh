#!/bin/bash
# A/B of engine library variants on one box: bench.py with RAFTGPU_LIB = each variant, alternated.
# usage: LIBS="build_variants/a.so build_variants/b.so" bash scripts/ab_lib.sh [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in $LIBS; do
    tag=$(basename $lib .so)_$rep
    timeout -k 10 ${AB_TIMEOUT:-150} env RAFTGPU_LIB=$PWD/$lib python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_$tag.log 2>&1 || { tail -5 gpurun_out/ab_$tag.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab_$tag.log').read().strip().splitlines()[-1])
print('$tag', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()})"
  done
done
