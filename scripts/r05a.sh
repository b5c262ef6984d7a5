set -o pipefail
mkdir -p gpurun_out
STEPS="smoke tests bench launch2" TAILN=6 bash scripts/gpu_round.sh
