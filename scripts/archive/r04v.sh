set -o pipefail
export TMPDIR=/tmp
for v in 1 1000003; do
mkdir -p gpurun_out/r04v_$v
RAFTGPU_POOL_PERM=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04v_$v/kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04v_$v/run.log 2>&1 || exit 1
python3 - $v <<'PY'
import csv,glob,sys,json
v=sys.argv[1]
rows=[]
for f in glob.glob(f'gpurun_out/r04v_{v}/kt/**/*kernel_trace.csv',recursive=True):
    rows+=list(csv.DictReader(open(f)))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
d=[round((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3) for r in rows if 'bulk_kernel' in r['Kernel_Name']]
print('perm', v, 'bulk', d[:50])
b=json.loads(open(f'gpurun_out/r04v_{v}/run.log').read().strip().splitlines()[-1])
print('perm', v, 'ms_per_step', round(b['ms_per_step'],4), 'untimed', round(b['ms_per_step_without_timing_events'],4))
PY
done
