# The r05 shapes re-measured with the settled bench (settle_ticks before warm-up): C5, C2, C2 metadata-only,
# and the one-rank rehearsals of the N > 1 step.
set -o pipefail
mkdir -p gpurun_out
line() {  # line NAME ARGS...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/r05w_$n.log 2>&1 || { tail -5 gpurun_out/r05w_$n.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r05w_$n.log') if l.startswith('{')][-1])
print('$n', round(d['ms_per_step'],4), 'untimed', round(d['ms_per_step_without_timing_events'],4), {k: round(v,4) for k,v in d['kernels_ms'].items()}, 'frac', round(d['roofline']['frac'],3), 'settle', d.get('settle_ticks'))"
}
line c5 --groups 1048576 --entries 1 --steps 10 --warmup 3
line c2 --groups 4096 --steps 100 --warmup 10
line c2p0 --groups 4096 --payload 0 --steps 100 --warmup 10
line rehearse_torch --wire-all --placement spread --steps 10 --warmup 3
line rehearse_c --wire-all --placement spread --exchange c --steps 10 --warmup 3
