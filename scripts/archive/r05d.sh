set -o pipefail
mkdir -p gpurun_out
STEPS="smoke tests bench" TAILN=4 bash scripts/gpu_round.sh || exit 1
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench.log') if l.startswith('{')][-1])
e=d['e2e_with_apply']; print('bench', round(d['value']/1e6,2), 'M; e2e', round(e['ms_per_step'],2), 'ms', e['schedules_ms_per_step'], 'bytes', e['bytes_per_step'], 'hand_off', round(e['hand_off']['ms_per_step'],2), 'apply', d['apply_copyback'])"
