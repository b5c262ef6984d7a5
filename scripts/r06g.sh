#!/bin/bash
# r06g: the page-pool step inside control_fastfb_kernel; the small-engine control kernels reload their
# parameter fields and fall back to the SLIM full step. GPU suite, then C2 / C2 P 0 against the
# hoisted build (ab/hoist.so: -DRG_CTL_RELOAD_LAT=0 -DRG_FB_SLIM=false), alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06g_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r06g_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r06g_gpu_tests.log
line() {  # line NAME LIB ARGS...
  local n=$1 lib=$2; shift 2
  RAFTGPU_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/r06g_$n.log 2>&1 || { tail -5 gpurun_out/r06g_$n.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06g_$n.log') if l.startswith('{')][-1])
print('$n', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, 'errs', d['replicas_with_invariant_errors'], 'resident', (d.get('graph') or {}).get('resident', {}).get('ms_per_step'))"
}
P=$PWD/raftd_amd/libraftgpu.so H=$PWD/ab/hoist.so
for i in 1 2; do
  line c2_new$i $P --groups 4096 --steps 100 --warmup 10
  line c2_hoist$i $H --groups 4096 --steps 100 --warmup 10
  line c2p0_new$i $P --groups 4096 --payload 0 --steps 100 --warmup 10
  line c2p0_hoist$i $H --groups 4096 --payload 0 --steps 100 --warmup 10
done
