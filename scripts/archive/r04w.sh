set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for v in 1 1000003; do RAFTGPU_POOL_PERM=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04w_$v.json 2>&1 || exit 1; python3 -c "
import json; d=json.loads(open('gpurun_out/r04w_$v.json').read().strip().splitlines()[-1]); print('perm $v', round(d['ms_per_step'],4), round(d['ms_per_step_without_timing_events'],4), round(d['roofline']['kernel_ms'],4), round(d['value']/1e6,2))"; done; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_configs.py tests/test_gpu_propose.py tests/test_gpu_snapshot.py > gpurun_out/r04w_tests.log 2>&1 || { tail -20 gpurun_out/r04w_tests.log; exit 1; }
tail -1 gpurun_out/r04w_tests.log
