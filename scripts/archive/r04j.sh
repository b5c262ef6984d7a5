set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_robust.py tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_kat.py tests/test_gpu_membership.py > gpurun_out/r04j_gpu_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r04j_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04j_gpu_tests.log
RAFTGPU_CTL_FB=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_gpu_membership.py > gpurun_out/r04j_gpu_tests_fb0.log 2>&1 || { echo fb0 tests failed; tail -30 gpurun_out/r04j_gpu_tests_fb0.log; exit 1; }
tail -1 gpurun_out/r04j_gpu_tests_fb0.log
VAR=RAFTGPU_CTL_FB VALS="1 0" bash scripts/ab_env.sh --groups 4096 --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04j_ab_fb_c2.txt || exit 1
VAR=RAFTGPU_CTL_FB VALS="1 0" bash scripts/ab_env.sh --groups 4096 --payload 0 --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04j_ab_fb_c2p0.txt || exit 1
VAR=RAFTGPU_CTL_FB VALS="1 0" bash scripts/ab_env.sh --groups 16384 --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04j_ab_fb_16k.txt || exit 1
timeout -k 10 200 python bench.py --groups 4096 --payload 0 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04j_c2p0.json 2>&1 || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/r04j_c2p0.json').read().strip().splitlines()[-1]); print('c2p0 tick', d['ms_per_step'], 'graph', d.get('graph',{}).get('ms_per_step'), 'resident', d.get('graph',{}).get('resident',{}).get('ms_per_step'))"
timeout -k 10 120 python scripts/ctl_profile.py abv/prof.so 4096 > gpurun_out/r04j_ctlprof_c2.txt 2>&1; cat gpurun_out/r04j_ctlprof_c2.txt
