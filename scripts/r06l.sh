#!/bin/bash
# r06l: the final build's kernel timelines of the small shapes (C2 P 256 and P 0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for shape in "c2:--groups 4096" "c2p0:--groups 4096 --payload 0"; do
  n=${shape%%:*}; args=${shape#*:}
  OUT=gpurun_out/prof_r06l_$n; rm -rf $OUT; mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace -- python3 bench.py $args --steps 100 --warmup 10 --no-cpu-baseline > $OUT/ktrace.log 2>&1 || { tail -5 $OUT/ktrace.log; exit 1; }
  f=$(find $OUT/ktrace -name "*kernel_trace.csv" | head -1)
  skip=$(python3 -c "
import json
d = json.loads([l for l in open('$OUT/ktrace.log') if l.startswith('{')][-1])
print(6 + d.get('settle_ticks', 0) + max(d['warmup'], 1))")
  echo "== $n (skip $skip)"
  python3 scripts/tick_timeline.py $f $skip 100 | tee $OUT/timeline.txt
done
