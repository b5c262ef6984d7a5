set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests > gpurun_out/gpu_tests_r04e.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_r04e.log; [ $rc -eq 0 ] || exit 1
VAR=RAFTGPU_CTL_FAST VALS="1 0" bash scripts/ab_env.sh --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04e_ab_fast_64k.txt || exit 1
VAR=RAFTGPU_CTL_FAST VALS="1 0" AB_TIMEOUT=300 bash scripts/ab_env.sh --groups 1048576 --entries 1 --steps 10 --warmup 3 2>&1 | tee gpurun_out/r04e_ab_fast_c5.txt || exit 1
VAR=RAFTGPU_CTL_FAST VALS="1 0" bash scripts/ab_env.sh --groups 4096 --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04e_ab_fast_c2.txt || exit 1
VAR=RAFTGPU_CTL_FAST VALS="1 0" bash scripts/ab_env.sh --groups 4096 --payload 0 --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04e_ab_fast_c2p0.txt
