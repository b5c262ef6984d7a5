set -o pipefail
mkdir -p gpurun_out
LIBS="abv/head2.so raftd_amd/libraftgpu.so" bash scripts/ab_lib.sh --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04m_ab_events.txt || exit 1
for L in abv/head2.so raftd_amd/libraftgpu.so; do timeout -k 10 200 env RAFTGPU_LIB=$PWD/$L python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04m_$(basename $L .so).json 2>&1 || exit 1; python3 -c "
import json; d=json.loads(open('gpurun_out/r04m_$(basename $L .so).json').read().strip().splitlines()[-1]); print('$L', d['ms_per_step'], d['ms_per_step_without_timing_events'], d['roofline']['kernel_ms'], d['value'])"; done
