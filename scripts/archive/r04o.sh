set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for v in 0 1; do timeout -k 10 200 env BENCH_PROBE_FIRST=$v python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04o_pf$v.json 2>&1 || exit 1; python3 -c "
import json; d=json.loads(open('gpurun_out/r04o_pf$v.json').read().strip().splitlines()[-1]); print('probe_first$v', round(d['ms_per_step'],4), round(d['ms_per_step_without_timing_events'],4), round(d['roofline']['kernel_ms'],4), round(d['graph']['ms_per_step'],4), round(d['roofline']['box_copy_ceiling_GBps']))"; done; done
LIBS="raftd_amd/libraftgpu.so abv/su8.so abv/su2.so" AB_TIMEOUT=300 bash scripts/ab_lib.sh --groups 1048576 --entries 1 --steps 10 --warmup 3 2>&1 | tee gpurun_out/r04o_ab_smallu_c5.txt || exit 1
