#!/bin/bash
# r06h: twin copies in bulk_kernel (R = 3: one read and CRC of a leader batch for both followers).
# The twin parity test and the GPU suite, then the 64K x 3 headline and C2 against the no-twin build
# (ab/notwin.so: -DRG_BULK_NO_TWIN), alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_twin.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r06h_twin_test.log 2>&1 || { tail -40 gpurun_out/r06h_twin_test.log; exit 1; }
tail -4 gpurun_out/r06h_twin_test.log
line() {  # line NAME LIB ARGS...
  local n=$1 lib=$2; shift 2
  RAFTGPU_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/r06h_$n.log 2>&1 || { tail -5 gpurun_out/r06h_$n.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06h_$n.log') if l.startswith('{')][-1])
r=d['roofline']
print('$n', round(d['ms_per_step'],4), round(d['value']/1e6,2), {k: round(v,4) for k,v in d['kernels_ms'].items()}, 'alg GB', round(r.get('algorithmic_bytes_per_launch',0)/1e9,3), 'frac', round(r['frac'],3), 'errs', d['replicas_with_invariant_errors'], 'twin', d['roofline'].get('tick_counts',{}).get('twin_entries'))"
}
P=$PWD/raftd_amd/libraftgpu.so N=$PWD/ab/notwin.so
for i in 1 2; do
  line head_twin$i $P --steps 20 --warmup 5
  line head_notwin$i $N --steps 20 --warmup 5
  line c2_twin$i $P --groups 4096 --steps 100 --warmup 10
  line c2_notwin$i $N --groups 4096 --steps 100 --warmup 10
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06h_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r06h_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r06h_gpu_tests.log
