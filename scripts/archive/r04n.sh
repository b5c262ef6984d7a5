set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for v in 0 1; do timeout -k 10 200 env RAFTGPU_POOL_TOUCH=$v python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04n_touch$v.json 2>&1 || exit 1; python3 -c "
import json; d=json.loads(open('gpurun_out/r04n_touch$v.json').read().strip().splitlines()[-1]); print('touch$v', round(d['ms_per_step'],4), round(d['ms_per_step_without_timing_events'],4), round(d['roofline']['kernel_ms'],4), round(d['graph']['ms_per_step'],4))"; done; done
