set -o pipefail
mkdir -p gpurun_out
VAR=RAFTGPU_BULK_WG VALS="4 3" bash scripts/ab_env.sh --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04x_ab_bulkwg_64k.txt || exit 1
VAR=RAFTGPU_BULK_WG VALS="4 3" bash scripts/ab_env.sh --steps 20 --warmup 5 2>&1 | tee -a gpurun_out/r04x_ab_bulkwg_64k.txt || exit 1
VAR=RAFTGPU_BULK_WG VALS="4 3" bash scripts/ab_env.sh --groups 4096 --steps 20 --warmup 5 2>&1 | tee gpurun_out/r04x_ab_bulkwg_c2.txt || exit 1
