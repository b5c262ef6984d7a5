# Head-page rows (bulk_small_kernel's page ids from coalesced rows instead of a page-table line per
# entry): correctness first (soak configurations, C5 and parity tests), then the C5 A/B against the
# page-table build (diag/nohp.so) and the 64K x 3 line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_soak.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_propose.py tests/test_gpu_compact.py tests/test_gpu_wal.py > gpurun_out/r05aa_tests.log 2>&1 || { tail -20 gpurun_out/r05aa_tests.log; exit 1; }
tail -1 gpurun_out/r05aa_tests.log
timeout -k 10 300 python -u scripts/soak.py 120 7000 > gpurun_out/r05aa_soak.log 2>&1 || { tail -5 gpurun_out/r05aa_soak.log; exit 1; }
tail -1 gpurun_out/r05aa_soak.log
LIBS="raftd_amd/libraftgpu.so diag/nohp.so" AB_TIMEOUT=300 bash scripts/ab_lib.sh --groups 1048576 --entries 1 --steps 10 --warmup 3 || exit 1
LIBS="raftd_amd/libraftgpu.so diag/nohp.so" bash scripts/ab_lib.sh --steps 20 --warmup 5 || exit 1
