#!/bin/bash
# Bench each experimental library in build_variants/ (RAFTGPU_LIB) plus the product build.
# usage: bash scripts/ablate.sh [variant ...]   (default: every build_variants/*.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
vs=("$@"); [ ${#vs[@]} -eq 0 ] && vs=($(ls build_variants/*.so 2>/dev/null | xargs -n1 basename | sed 's/\.so$//'))
run() {
  timeout -k 10 300 env $2 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/abl_$1.log 2>&1 || { echo "$1 FAILED"; tail -5 gpurun_out/abl_$1.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/abl_$1.log').read().strip().splitlines()[-1]); print('$1', round(d['ms_per_step'],3), 'dev', round(d['device_ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()}, 'frac', round(d['roofline']['frac'],3))"
}
run product ""
for v in "${vs[@]}"; do run $v RAFTGPU_LIB=$PWD/build_variants/$v.so; done
run product_again ""
