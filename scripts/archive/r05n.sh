# The region to self packed in place (rg_wire_pack_at; no self copy): the wire / cluster / exchange GPU
# tests, then the N = 1 rehearsals of the N > 1 step (torch exchange and the C exchange).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cluster.py tests/test_abi.py tests/test_gpu_configs.py > gpurun_out/r05n_tests.log 2>&1 || { tail -20 gpurun_out/r05n_tests.log; exit 1; }
tail -1 gpurun_out/r05n_tests.log
STEPS="rehearse_nccl rehearse_c" TAILN=4 bash scripts/gpu_round.sh || exit 1
for f in rehearse_nccl rehearse_c; do python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1])
print('$f', round(d['ms_per_step'],3), 'ctl', round(d['kernels_ms']['control_kernel'],3), 'bulk', round(d['kernels_ms']['bulk_kernel'],3), 'slow', d['control_fast_path']['slow_replicas_last_tick'], 'drops', d['drops_total'])"; done
