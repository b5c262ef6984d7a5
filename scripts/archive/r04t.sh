set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_robust.py tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_membership.py tests/test_gpu_snapshot.py > gpurun_out/r04t_gpu_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r04t_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04t_gpu_tests.log
for rep in 1 2; do for L in abv/head2.so raftd_amd/libraftgpu.so; do timeout -k 10 200 env RAFTGPU_LIB=$PWD/$L python bench.py --groups 4096 --payload 0 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04t_c2p0.json 2>&1 || exit 1; python3 -c "
import json; d=json.loads(open('gpurun_out/r04t_c2p0.json').read().strip().splitlines()[-1]); print('$L', 'tick', round(d['ms_per_step'],4), 'graph', round(d['graph']['ms_per_step'],4), 'resident', round(d['graph']['resident']['ms_per_step'],4))"; done; done
LIBS="abv/head2.so raftd_amd/libraftgpu.so" bash scripts/ab_lib.sh --groups 4096 --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04t_ab_c2.txt || exit 1
