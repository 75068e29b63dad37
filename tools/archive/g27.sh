set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --matrix lj --steps 2 --warmup 1 --no-cpu-baseline --tiled 0 > gpurun_out/g27_lj.json 2>gpurun_out/g27_lj.err; rc=$?; tail -3 gpurun_out/g27_lj.err; [ $rc -eq 0 ] || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/g27_lj.json'));print('lj full',d['ms_per_step'],d['value'],d['config']['path'],d['config'].get('row_blocks'))"
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/g27tiled -o run -- python3 $GRAFT_REPO_ROOT/tools/tiled_time.py webbase 3 > $GRAFT_REPO_ROOT/gpurun_out/g27tiled.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT; tail -2 gpurun_out/g27tiled.log
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/g27tiled/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:22]:
    print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:9.1f}')
PY
