set -o pipefail
mkdir -p gpurun_out
STEPS="tests" TAILN=3 bash scripts/gpu_round.sh || exit 1
C5="--groups 1048576 --entries 1 --steps 10 --warmup 3 --no-cpu-baseline"
timeout -k 10 300 python bench.py $C5 > gpurun_out/r05f_c5_bench.log 2>&1 || { tail -5 gpurun_out/r05f_c5_bench.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r05f_c5_bench.log') if l.startswith('{')][-1])
print('c5 bench', round(d['ms_per_step'],3), d['kernels_ms'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r05f_bench.log 2>&1 || { tail -5 gpurun_out/r05f_bench.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r05f_bench.log') if l.startswith('{')][-1])
print('bench', round(d['value']/1e6,2), round(d['ms_per_step'],3), d['kernels_ms'], round(d['roofline']['frac'],3))"
bash scripts/r05e.sh
