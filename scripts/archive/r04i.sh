set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_robust.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_digest.py > gpurun_out/r04i_gpu_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r04i_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04i_gpu_tests.log
LIBS="abv/head.so raftd_amd/libraftgpu.so" bash scripts/ab_lib.sh --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04i_ab_64k.txt || exit 1
LIBS="abv/head.so raftd_amd/libraftgpu.so" bash scripts/ab_lib.sh --groups 4096 --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04i_ab_c2.txt || exit 1
LIBS="abv/head.so raftd_amd/libraftgpu.so" bash scripts/ab_lib.sh --groups 4096 --payload 0 --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04i_ab_c2p0.txt || exit 1
LIBS="abv/head.so raftd_amd/libraftgpu.so" AB_TIMEOUT=300 bash scripts/ab_lib.sh --groups 1048576 --entries 1 --steps 10 --warmup 3 2>&1 | tee gpurun_out/r04i_ab_c5.txt || exit 1
timeout -k 10 120 python scripts/ctl_profile.py abv/prof.so > gpurun_out/r04i_ctlprof.txt 2>&1; cat gpurun_out/r04i_ctlprof.txt
bash scripts/sq_counters.sh r04i; tail -2 gpurun_out/sq_r04i/run.log
