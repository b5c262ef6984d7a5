set -o pipefail
mkdir -p gpurun_out
STEPS="tests launch2 rehearse_nccl rehearse_c" TAILN=4 bash scripts/gpu_round.sh || exit 1
for f in launch2 rehearse_nccl rehearse_c; do python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), 'ctl', round(d['kernels_ms']['control_kernel'],3), 'bulk', round(d['kernels_ms']['bulk_kernel'],3), 'slow', d['control_fast_path']['slow_replicas_last_tick'], 'drops', d['drops_total'])"; done
