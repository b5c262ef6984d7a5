set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04r
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04r/kt -- python3 bench.py --steps 20 --warmup 40 --no-cpu-baseline > gpurun_out/r04r/run.log 2>&1 || exit 1
python3 - <<'PY'
import csv,glob
rows=[]
for f in glob.glob('gpurun_out/r04r/kt/**/*kernel_trace.csv',recursive=True):
    rows+=list(csv.DictReader(open(f)))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
for name in ('bulk_kernel','control_fast','pool_kernel'):
    d=[round((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3) for r in rows if name in r['Kernel_Name']]
    print(name, len(d), d[:70])
PY
