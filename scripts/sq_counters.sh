#!/bin/bash
# Instruction mix and wait cycles of the tick kernels (one rocprofv3 PMC pass, SQ block only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/sq_$1; shift
rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM} \
  --output-format csv -d $OUT -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline "$@" > $OUT/run.log 2>&1
rc=$?
python3 - $OUT <<'PY'
import csv, glob, sys, collections
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r["Kernel_Name"]
    k = ("control_fast" if "control_fast_kernel" in k else "control_slow" if "control_slow_kernel" in k
         else "control" if "control_kernel" in k else "bulk" if "bulk_kernel" in k else None)
    if k:
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    m = {c: sorted(v)[len(v) // 2] for c, v in d.items()}  # median over dispatches
    w = m.get("SQ_WAVES", 1) or 1
    print(k, {c: round(v / w, 1) for c, v in sorted(m.items())}, "per wave; waves", w)
PY
exit $rc
