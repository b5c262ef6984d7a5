#!/bin/bash
# r06k: what control(t+1) beside bulk(t) would give — the RG_OVERLAP ablation (bulk on a second stream;
# NOT the product: it keeps the three hazards DESIGN §3 names, which these steady-state shapes do not
# hit) against the product, on the headline, C5 and C2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
line() {  # line NAME LIB ARGS...
  local n=$1 lib=$2; shift 2
  RAFTGPU_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/r06k_$n.log 2>&1 || { tail -5 gpurun_out/r06k_$n.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06k_$n.log') if l.startswith('{')][-1])
print('$n', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, 'errs', d['replicas_with_invariant_errors'], 'commits', d['commits_measured_per_step'], '/', d['commits_expected_per_step'])"
}
P=$PWD/raftd_amd/libraftgpu.so O=$PWD/ab/overlap.so
for i in 1 2; do
  line head_prod$i $P --steps 20 --warmup 5
  line head_ovl$i $O --steps 20 --warmup 5
  line c2_prod$i $P --groups 4096 --steps 100 --warmup 10
  line c2_ovl$i $O --groups 4096 --steps 100 --warmup 10
done
line c5_prod $P --groups 1048576 --entries 1 --steps 10 --warmup 3
line c5_ovl $O --groups 1048576 --entries 1 --steps 10 --warmup 3
