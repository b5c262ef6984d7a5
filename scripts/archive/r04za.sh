set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_cluster.py > gpurun_out/r04za_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r04za_tests.log; exit 1; }
tail -1 gpurun_out/r04za_tests.log
for w in 5 30; do for args in "--exchange c --sizing fixed" "--exchange c --sizing exact"; do RAFTGPU_WIRE_SIZING=$(echo $args | awk '{print $NF}') timeout -k 10 300 python bench.py --placement spread --wire-all --no-cpu-baseline --steps 10 --warmup $w $args > gpurun_out/r04za_rehearse.json 2>&1 || { tail -5 gpurun_out/r04za_rehearse.json; exit 1; }; python3 -c "
import json; d=json.loads(open('gpurun_out/r04za_rehearse.json').read().strip().splitlines()[-1]); x=d['exchange']; print('warmup $w $args', round(d['ms_per_step'],3), x['transport'][:70], 'drops', d['drops_total'])" | tee -a gpurun_out/r04za_sizing.txt; done; done
