set -o pipefail
STEPS="smoke tests" bash scripts/gpu_round.sh && bash scripts/c2_probe.sh && timeout -k 10 120 python scripts/ctl_profile.py build_variants/ctlprof.so 4096
