set -e
mkdir -p gpurun_out/g11
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/g11/stats -o run -- python3 $GRAFT_REPO_ROOT/tools/tiled_time.py webbase 3 > $GRAFT_REPO_ROOT/gpurun_out/g11/log 2>&1
cd $GRAFT_REPO_ROOT
grep "t_tile" gpurun_out/g11/log
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/g11/stats/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:30]:
    print(f'{r["Name"][:80]:80s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:9.1f}')
PY
