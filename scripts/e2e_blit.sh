#!/bin/bash
# e2e_with_apply (tick + async copy-back of one node's applied entries) against the number of
# workgroups the runtime's blit (copy) kernels may use: DEBUG_CLR_LIMIT_BLIT_WG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in ${WGS:-0 8 32}; do
  if [ "$w" = 0 ]; then unset DEBUG_CLR_LIMIT_BLIT_WG; else export DEBUG_CLR_LIMIT_BLIT_WG=$w; fi
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/e2e_wg$w.log 2>&1 || { tail -5 gpurun_out/e2e_wg$w.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/e2e_wg$w.log').read().strip().splitlines()[-1]); e=d['e2e_with_apply']; a=d['apply_copyback']
print('blit_wg $w', 'tick', round(d['ms_per_step'],3), 'e2e', round(e['ms_per_step'],2), 'ms', round(e['pcie_GBps'],1), 'GB/s; sync copy-back', round(a['ms'],1), 'ms', round(a['GBps'],1), 'GB/s')"
done
