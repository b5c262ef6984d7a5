set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_cluster.py tests/test_nodehost.py tests/test_abi.py > gpurun_out/r04y_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r04y_tests.log; exit 1; }
tail -1 gpurun_out/r04y_tests.log
for args in "--exchange c" "--sizing exact" "--sizing fixed"; do timeout -k 10 300 python bench.py --placement spread --wire-all --no-cpu-baseline --steps 10 --warmup 5 $args > gpurun_out/r04y_rehearse.json 2>&1 || { tail -5 gpurun_out/r04y_rehearse.json; exit 1; }; python3 -c "
import json; d=json.loads(open('gpurun_out/r04y_rehearse.json').read().strip().splitlines()[-1]); x=d['exchange']; print('$args', round(d['ms_per_step'],3), x['transport'][:60], round(x['bytes_sent_per_step_max_rank']/1e6,1), 'drops', d['drops_total'])"; done
