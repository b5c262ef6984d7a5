# S_LAST_TERM (the term of entry `last` as a state row, no ring read at the start of the step):
# correctness (parity, KAT, configs, soak), then A/B against the ring read (diag/ltring.so) at C5 and 64K x 3.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_configs.py tests/test_gpu_soak.py tests/test_gpu_wal.py tests/test_gpu_membership.py tests/test_gpu_read_index.py > gpurun_out/r05ai_tests.log 2>&1 || { tail -20 gpurun_out/r05ai_tests.log; exit 1; }
tail -1 gpurun_out/r05ai_tests.log
LIBS="raftd_amd/libraftgpu.so diag/ltring.so" AB_TIMEOUT=300 bash scripts/ab_lib.sh --groups 1048576 --entries 1 --steps 10 --warmup 3 || exit 1
LIBS="raftd_amd/libraftgpu.so diag/ltring.so" bash scripts/ab_lib.sh --steps 20 --warmup 5 || exit 1
