#!/bin/bash
# r06m: C2 with the latency build's followers prefetching their next inbox header (ab/latpipe.so,
# -DRG_CTL_LAT_FOLLOWER_PIPE) against the product, alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
line() {  # line NAME LIB ARGS...
  local n=$1 lib=$2; shift 2
  RAFTGPU_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/r06m_$n.log 2>&1 || { tail -5 gpurun_out/r06m_$n.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06m_$n.log') if l.startswith('{')][-1])
g=d.get('graph') or {}
print('$n', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, 'errs', d['replicas_with_invariant_errors'], 'resident', (g.get('resident') or {}).get('ms_per_step'))"
}
P=$PWD/raftd_amd/libraftgpu.so A=$PWD/ab/latpipe.so
for i in 1 2; do
  line c2p0_prod$i $P --groups 4096 --payload 0 --steps 100 --warmup 10
  line c2p0_pipe$i $A --groups 4096 --payload 0 --steps 100 --warmup 10
  line c2_prod$i $P --groups 4096 --steps 100 --warmup 10
  line c2_pipe$i $A --groups 4096 --steps 100 --warmup 10
done
