set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for L in abv/none.so abv/nodeep.so abv/nolat.so raftd_amd/libraftgpu.so; do timeout -k 10 200 env RAFTGPU_LIB=$PWD/$L python bench.py --groups 4096 --payload 0 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04u_c2p0.json 2>&1 || exit 1; python3 -c "
import json; d=json.loads(open('gpurun_out/r04u_c2p0.json').read().strip().splitlines()[-1]); print('$L', 'tick', round(d['ms_per_step'],4), 'ctl', round(d['kernels_ms']['control_kernel'],4), 'resident', round(d['graph']['resident']['ms_per_step'],4))"; done; done
