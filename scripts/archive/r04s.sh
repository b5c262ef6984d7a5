set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests > gpurun_out/r04s_gpu_tests.log 2>&1 || { echo suite failed; tail -30 gpurun_out/r04s_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04s_gpu_tests.log
bash scripts/r04r.sh
