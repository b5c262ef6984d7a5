set -o pipefail
mkdir -p gpurun_out
STEPS="smoke tests bench launch2 rehearse_nccl rehearse_c" TAILN=6 bash scripts/gpu_round.sh
