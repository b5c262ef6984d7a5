#!/bin/bash
# bulk_kernel grid (blocks) at a shape: RAFTGPU_BULK_GRID overrides the engine's choice (0 = default).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for gsz in ${GRIDS:-0 512 1536 2048}; do
  if [ "$gsz" = 0 ]; then unset RAFTGPU_BULK_GRID; else export RAFTGPU_BULK_GRID=$gsz; fi
  timeout -k 10 120 python bench.py ${SHAPE:---groups 4096 --steps 100 --warmup 10} --no-cpu-baseline > gpurun_out/grid_$gsz.log 2>&1 || { tail -5 gpurun_out/grid_$gsz.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/grid_$gsz.log').read().strip().splitlines()[-1])
print('grid $gsz', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, 'frac', round(d['roofline']['frac'],3))"
done
