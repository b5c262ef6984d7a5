# The full step's load batch (RG_CTL_FULL_BATCH 2, no VGPR spills) against r05's 8 (diag/cb8.so):
# election storm (most replicas take the full step), C2 (fastfb) and the 64K x 3 line.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in raftd_amd/libraftgpu.so diag/cb8.so; do
    echo "$lib storm $(timeout -k 10 200 env RAFTGPU_LIB=$PWD/$lib python scripts/storm_probe.py 2>&1 | tail -1)"
  done
done
LIBS="raftd_amd/libraftgpu.so diag/cb8.so" bash scripts/ab_lib.sh --groups 4096 --steps 100 --warmup 10 || exit 1
LIBS="raftd_amd/libraftgpu.so diag/cb8.so" bash scripts/ab_lib.sh --groups 4096 --payload 0 --steps 100 --warmup 10 || exit 1
