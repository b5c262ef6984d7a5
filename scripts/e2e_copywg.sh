#!/bin/bash
# The overlapped copy-back (rg_apply_async: a copy kernel streams the gathered batch into host-mapped
# memory beside the next ticks) against the number of copy workgroups: fewer host writes in flight
# may stall the concurrent tick kernels less (r03b trace: with 32 workgroups control ran 3-4 ms and
# bulk 15 ms beside the copy, instead of 0.13 / 1.27 ms).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wg in ${WGS:-2 4 8 16 32}; do
  RAFTGPU_COPY_WG=$wg timeout -k 10 300 python bench.py --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/e2e_wg$wg.log 2>&1 || { tail -5 gpurun_out/e2e_wg$wg.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/e2e_wg$wg.log').read().strip().splitlines()[-1]);e=d['e2e_with_apply']
print('wg $wg overlapped ms', round(e['ms_per_step'],2), 'GB/s', round(e['pcie_GBps'],1), 'serial ms', round(e['serial']['ms_per_step'],2), 'GB/s', round(e['serial']['pcie_GBps'],1), 'tick ms', round(d['ms_per_step'],4))"
done
