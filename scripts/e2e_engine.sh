#!/bin/bash
# e2e_with_apply against the runtime's copy engine choice (GPU_BLIT_ENGINE_TYPE, HSA_ENABLE_SDMA).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
env | grep -iE "sdma|blit" || true
for cfg in "${CFGS[@]:-base}"; do :; done
run() {  # run TAG VAR=VAL...
  local tag=$1; shift
  timeout -k 10 200 env "$@" python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/e2e_$tag.log 2>&1 || { tail -5 gpurun_out/e2e_$tag.log; return 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/e2e_$tag.log').read().strip().splitlines()[-1]); e=d['e2e_with_apply']; a=d['apply_copyback']
print('$tag', 'tick', round(d['ms_per_step'],3), 'e2e', round(e['ms_per_step'],2), 'ms', round(e['pcie_GBps'],1), 'GB/s; sync copy-back', round(a['ms'],1), 'ms', round(a['GBps'],1), 'GB/s')"
}
run sdma1 HSA_ENABLE_SDMA=1 && run blit1 GPU_BLIT_ENGINE_TYPE=1 && run blit2 GPU_BLIT_ENGINE_TYPE=2 && run blit3 GPU_BLIT_ENGINE_TYPE=3
