#!/bin/bash
# r06 final build (speculated parameter-block chunks), call C: smoke, the GPU suite, the default bench
# line, and the shape lines (C5, C2, C2 P 0, the wire rehearsal through rg_wire_exchange).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BENCH_ARGS=" " STEPS="smoke tests bench" bash scripts/gpu_round.sh || exit 1
line() {  # line NAME ARGS...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/r06_final_$n.log 2>&1 || { tail -5 gpurun_out/r06_final_$n.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r06_final_$n.log') if l.startswith('{')][-1])
x=d.get('exchange') or {}
g=d.get('graph') or {}
print('$n', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, 'frac', round(d['roofline']['frac'],3), 'errs', d['replicas_with_invariant_errors'], 'bound_ms', x.get('bound_ms'), 'resident', (g.get('resident') or {}).get('ms_per_step'))"
}
line c5 --groups 1048576 --entries 1 --steps 10 --warmup 3
line c2 --groups 4096 --steps 100 --warmup 10
line c2p0 --groups 4096 --payload 0 --steps 100 --warmup 10
line rehearse_c --wire-all --placement spread --exchange c --steps 10 --warmup 3
