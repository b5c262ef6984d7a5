#!/bin/bash
# r06i: bulk_kernel at occupancy 5 (ab/pad.so: one more TileJobs field moves the non-MJ kernels from
# 97 / 102 to 87 / 91 VGPRs) against the product (occupancy 4): the headline, C2, the wire rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
line() {  # line NAME LIB ARGS...
  local n=$1 lib=$2; shift 2
  RAFTGPU_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/r06i_$n.log 2>&1 || { tail -5 gpurun_out/r06i_$n.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06i_$n.log') if l.startswith('{')][-1])
r=d['roofline']
print('$n', round(d['ms_per_step'],4), round(d['value']/1e6,2), {k: round(v,4) for k,v in d['kernels_ms'].items()}, 'frac', round(r['frac'],3), 'errs', d['replicas_with_invariant_errors'])"
}
P=$PWD/raftd_amd/libraftgpu.so A=$PWD/ab/pad.so
for i in 1 2 3; do
  line head_prod$i $P --steps 20 --warmup 5
  line head_pad$i $A --steps 20 --warmup 5
done
for i in 1 2; do
  line c2_prod$i $P --groups 4096 --steps 100 --warmup 10
  line c2_pad$i $A --groups 4096 --steps 100 --warmup 10
  line reh_prod$i $P --wire-all --placement spread --exchange c --steps 10 --warmup 3
  line reh_pad$i $A --wire-all --placement spread --exchange c --steps 10 --warmup 3
done
