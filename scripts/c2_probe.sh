#!/bin/bash
# A/B of the product library against build_variants/*.so at the 64K default, C2 (4,096 groups) and
# C2 metadata-only (P = 0) shapes; one line per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # run NAME ENV ARGS...
  local n=$1 env=$2; shift 2
  timeout -k 10 200 env $env python bench.py "$@" --no-cpu-baseline > gpurun_out/c2_$n.log 2>&1 || { tail -5 gpurun_out/c2_$n.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/c2_$n.log').read().strip().splitlines()[-1])
print('$n', '$*', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, round(d['roofline']['frac'],3))"
}
for v in product $(ls build_variants/*.so | grep -v ctlprof 2>/dev/null | xargs -n1 basename | sed 's/\.so$//') product; do
  env=""; [ $v != product ] && env=RAFTGPU_LIB=$PWD/build_variants/$v.so
  run $v "$env" --steps 20 --warmup 5
  run ${v}_c2 "$env" --groups 4096 --steps 100 --warmup 10
  run ${v}_c2p0 "$env" --groups 4096 --payload 0 --steps 100 --warmup 10
done
