#!/bin/bash
# bulk_kernel tile size at the C2 shape (4,096 x 3): RAFTGPU_BULK_TILE overrides the engine's choice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for t in ${TILES:-0 1 2 4 8 16}; do
  if [ "$t" = 0 ]; then unset RAFTGPU_BULK_TILE; else export RAFTGPU_BULK_TILE=$t; fi
  timeout -k 10 120 python bench.py ${SHAPE:---groups 4096 --steps 100 --warmup 10} --no-cpu-baseline > gpurun_out/tile_$t.log 2>&1 || { tail -5 gpurun_out/tile_$t.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/tile_$t.log').read().strip().splitlines()[-1])
print('tile $t', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, 'frac', round(d['roofline']['frac'],3))"
done
