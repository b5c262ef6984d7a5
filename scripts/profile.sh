#!/bin/bash
# Profile the bench's tick kernel on the GPU box: kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE in separate PMC passes (MI355X_MICROARCH.md: TCC slots cannot hold both).
# usage: bash scripts/profile.sh TAG [bench args...]
set -euo pipefail
TAG=$1; shift
ARGS="${@:---steps 10 --warmup 3 --no-cpu-baseline}"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace -- python3 bench.py $ARGS > $OUT/ktrace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -- python3 bench.py $ARGS > $OUT/write.log 2>&1
# the timed window starts after bring-up (6 ticks), the settle ticks and the warm-up: read from the bench line
HEAD_DEF=$(python3 -c "
import json
d = json.loads([l for l in open('$OUT/ktrace.log') if l.startswith('{')][-1])
print(6 + d.get('settle_ticks', 0) + max(d['warmup'], 1))")
SKIP_HEAD=${SKIP_HEAD:-$HEAD_DEF} PROFILES_DIR=$OUT python3 scripts/pmc_summary.py $TAG $OUT/ktrace $OUT/fetch $OUT/write ${LAST_N:-10} ${SKIP:-92}  # SKIP_HEAD = bring-up ticks (6) + settle + warm-up: the window is the timed ticks (SKIP, unused then = tick launches after the timed region: CONTROL_TIMING_STEPS (4) + the untimed repeat (steps) + the graph measurement (5 x 10) + two e2e_with_apply runs (overlapped, serial) of min(steps, 12) + the hand-off run of min(steps, 8); copy into profiles/ after the call
