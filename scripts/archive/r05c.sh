set -o pipefail
mkdir -p gpurun_out
C5="--groups 1048576 --entries 1 --steps 10 --warmup 3 --no-cpu-baseline"
timeout -k 10 300 python bench.py $C5 > gpurun_out/r05c_c5_bench.log 2>&1 || { tail -5 gpurun_out/r05c_c5_bench.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r05c_c5_bench.log') if l.startswith('{')][-1])
print('c5 bench', round(d['ms_per_step'],3), d['kernels_ms'], 'tick bytes', d['roofline']['tick_algorithmic_bytes'], 'bulk bytes', d['roofline']['algorithmic_bytes_per_launch'])"
bash scripts/profile.sh r05c_c5 $C5 || exit 1
bash scripts/sq_counters.sh r05c_c5 --groups 1048576 --entries 1 || exit 1
PMC="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU" bash scripts/sq_counters.sh r05c_c5b --groups 1048576 --entries 1 || exit 1
