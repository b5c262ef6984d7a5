#!/bin/bash
# bench.py at the other BASELINE.json shapes on one GPU (steady-state leaders; not the headline
# line): C2 4,096 x 3 (and P = 0), 64K x 3 P = 0, C3's shape co-located at 32K x 5 (64K x 5 at L 2,048 holds more live Cmds than one engine's 64-GiB page pool),
# C5's 1M x 3 at P = 256, L = 2,048 (the paged store, r03).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # run NAME ARGS...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/shape_$n.log 2>&1 || { tail -5 gpurun_out/shape_$n.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/shape_$n.log').read().strip().splitlines()[-1])
r=d['roofline']
print('$n', '$*', 'value', round(d['value']/1e6,2), 'M ms', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()},
      'bulkGBs', round(r['achieved']), 'frac', round(r['frac'],3), 'commits/s', round(d['commits_per_sec']/1e9,3), 'G err', d['replicas_with_invariant_errors'],
      'dev GB', round(d['device_bytes']/1e9,1))"
}
run c2 --groups 4096 --steps 100 --warmup 10
run c2p0 --groups 4096 --payload 0 --steps 100 --warmup 10
run m64p0 --payload 0 --steps 50 --warmup 10
run c3shape --replicas 5 --groups 32768 --steps 20 --warmup 5  # 32K x 5 = C3's 8,192 columns x 5 per GPU, four times over
run c5shape --groups 1048576 --entries 1 --steps 10 --warmup 3  # mean 1 entry per group per tick
