# A/B: the full step's parameter reloads (product: SGPR spills 456 -> 66) vs r04's hoisted loads
# (diag/hoist.so) vs reloads in the fast step too (diag/reload_fast.so): 64K x 3, C5 shape, C2.
set -o pipefail
mkdir -p gpurun_out
export LIBS="raftd_amd/libraftgpu.so diag/hoist.so diag/reload_fast.so"
echo "== 64K x 3"; bash scripts/ab_lib.sh --steps 20 --warmup 5 || exit 1
echo "== C5 shape"; AB_TIMEOUT=300 bash scripts/ab_lib.sh --groups 1048576 --entries 1 --steps 10 --warmup 3 || exit 1
echo "== C2"; bash scripts/ab_lib.sh --groups 4096 --steps 100 --warmup 10 || exit 1
echo "== C2 P0"; bash scripts/ab_lib.sh --groups 4096 --payload 0 --steps 100 --warmup 10 || exit 1
