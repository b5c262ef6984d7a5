set -o pipefail
mkdir -p gpurun_out
for w in 5 30 60; do timeout -k 10 200 python bench.py --steps 20 --warmup $w --no-cpu-baseline > gpurun_out/r04p_w$w.json 2>&1 || exit 1; python3 -c "
import json; d=json.loads(open('gpurun_out/r04p_w$w.json').read().strip().splitlines()[-1]); print('warmup $w', round(d['ms_per_step'],4), round(d['ms_per_step_without_timing_events'],4), round(d['roofline']['kernel_ms'],4), round(d['kernels_ms']['control_kernel'],4))"; done
