set -o pipefail
mkdir -p gpurun_out
T=tests/test_gpu_configs.py::test_c3_five_replicas_eight_ranks_full_size
PT="timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider -m gpu"
RAFTGPU_CTL_FAST=0 $PT $T > gpurun_out/r04g_full.log 2>&1 || { echo full failed; tail -2 gpurun_out/r04g_full.log; exit 1; }
echo full ok
$PT $T > gpurun_out/r04g_fast.log 2>&1 || { echo fast failed; tail -2 gpurun_out/r04g_fast.log; exit 1; }
echo fast ok
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests > gpurun_out/r04g_gpu_tests.log 2>&1 || { echo suite failed; tail -30 gpurun_out/r04g_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04g_gpu_tests.log
VAR=RAFTGPU_BULK_SMALL VALS="1 0" AB_TIMEOUT=300 bash scripts/ab_env.sh --groups 1048576 --entries 1 --steps 10 --warmup 3 2>&1 | tee gpurun_out/r04g_ab_small_c5.txt || exit 1
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --ingest --no-cpu-baseline > gpurun_out/r04g_ingest.json 2> gpurun_out/r04g_ingest.err || { tail -5 gpurun_out/r04g_ingest.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04g_ingest.json').read().strip().splitlines()[-1])['ingest']
print('ingest', {k: d[k] for k in ('ms_per_step','propose_ms_per_step','ingest_GBps')}, 'registered', {k: d['registered'][k] for k in ('ms_per_step','propose_ms_per_step','ingest_GBps')})"
LIBS="abv/head.so raftd_amd/libraftgpu.so abv/np.so abv/np3.so" bash scripts/ab_lib.sh --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04g_ab_64k.txt || exit 1
LIBS="abv/head.so raftd_amd/libraftgpu.so abv/np.so abv/np3.so" bash scripts/ab_lib.sh --groups 4096 --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04g_ab_c2.txt || exit 1
timeout -k 10 120 python scripts/ctl_profile.py abv/prof.so > gpurun_out/r04g_ctlprof.txt 2>&1; cat gpurun_out/r04g_ctlprof.txt
timeout -k 10 120 python scripts/ctl_profile.py abv/prof.so 4096 > gpurun_out/r04g_ctlprof_c2.txt 2>&1; cat gpurun_out/r04g_ctlprof_c2.txt
bash scripts/sq_counters.sh r04g; tail -2 gpurun_out/sq_r04g/run.log
