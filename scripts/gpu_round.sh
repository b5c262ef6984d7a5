#!/bin/bash
# One GPU call: smoke, the GPU test suite, the N=1 bench, an N=1 wire-all bench and a 2-rank gloo
# rehearsal of the N>1 bench path on the one GPU. Stops at the first failure / fault.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fault() { grep -q "HSA_STATUS_ERROR\|illegal memory access\|Memory access fault" "$1"; }
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  tail -${TAILN:-4} gpurun_out/$name.log
  if [ $rc -ne 0 ] || fault gpurun_out/$name.log; then echo "$name FAILED rc=$rc"; exit 1; fi
}
for what in ${STEPS:-smoke parity tests bench wire rehearse}; do
  case $what in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    parity) TAILN=3 step gpu_parity 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider ;;
    tests) TAILN=6 step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider ;;
    bench) step bench 400 python bench.py ${BENCH_ARGS:---cpu-seconds 10 --ingest} ;;
    profile) step profile 1000 bash scripts/profile.sh ${PTAG:-r03} ;;
    shapes) step shapes 600 bash scripts/shapes.sh ;;
    copywg) step copywg 900 bash scripts/e2e_copywg.sh ;;
    mj) echo "mj: retired (RAFTGPU_BULK_MULTIJOB is a build variant now: scripts/build_variant.sh -DRG_AB_BULK_MULTIJOB=0/1)"; exit 1 ;;
    rehearse_c) step rehearse_c 400 python bench.py --placement spread --wire-all --exchange c --no-cpu-baseline --steps 10 --warmup 3 ;;
    sdma) step sdma 300 env RAFTGPU_APPLY_SDMA=1 python bench.py --steps 12 --warmup 3 --no-cpu-baseline ;;
    wire) step bench_wire 400 python bench.py --wire-all --no-cpu-baseline ;;
    rehearse) step rehearse 400 env RAFTD_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --backend gloo --groups 8192 \
                --steps 5 --warmup 2 ;;
    rehearse_nccl) step rehearse_nccl 400 python bench.py --placement spread --wire-all --no-cpu-baseline \
                --steps 10 --warmup 3 ;;
    rehearse8) step rehearse8 500 env RAFTD_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
                --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 8 --backend gloo --groups 2048 \
                --steps 4 --warmup 2 ;;
    launch2) step launch2 600 python bench.py --gpus 2 --backend gloo --no-cpu-baseline --steps 5 --warmup 2 ;;
    rehearse1) step rehearse1 400 env RAFTD_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --backend gloo --groups 8192 \
                --steps 5 --warmup 2 --halves 1 ;;
  esac
done
echo ALL-OK
