#!/bin/bash
# r06j: C2's bulk tile (replicas per wave work item): the product's rule against fixed tiles of 1 and 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
line() {  # line NAME LIB ARGS...
  local n=$1 lib=$2; shift 2
  RAFTGPU_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/r06j_$n.log 2>&1 || { tail -5 gpurun_out/r06j_$n.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06j_$n.log') if l.startswith('{')][-1])
print('$n', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, 'frac', round(d['roofline']['frac'],3), 'errs', d['replicas_with_invariant_errors'])"
}
P=$PWD/raftd_amd/libraftgpu.so T1=$PWD/ab/tile1.so T2=$PWD/ab/tile2.so
for i in 1 2; do
  line c2_prod$i $P --groups 4096 --steps 100 --warmup 10
  line c2_tile1_$i $T1 --groups 4096 --steps 100 --warmup 10
  line c2_tile2_$i $T2 --groups 4096 --steps 100 --warmup 10
done
line c5_prod $P --groups 1048576 --entries 1 --steps 10 --warmup 3
