set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests > gpurun_out/gpu_tests_r04f.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_r04f.log; [ $rc -eq 0 ] || exit 1
LIBS="abv/head.so raftd_amd/libraftgpu.so abv/w3.so" bash scripts/ab_lib.sh --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04f_ab_64k.txt || exit 1
LIBS="abv/head.so raftd_amd/libraftgpu.so" AB_TIMEOUT=300 bash scripts/ab_lib.sh --groups 1048576 --entries 1 --steps 10 --warmup 3 2>&1 | tee gpurun_out/r04f_ab_c5.txt || exit 1
LIBS="abv/head.so raftd_amd/libraftgpu.so" bash scripts/ab_lib.sh --groups 4096 --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04f_ab_c2.txt || exit 1
timeout -k 10 120 python scripts/ctl_profile.py abv/prof.so > gpurun_out/r04f_ctlprof.txt 2>&1; cat gpurun_out/r04f_ctlprof.txt
bash scripts/sq_counters.sh r04f; cat gpurun_out/sq_r04f/run.log | tail -2
