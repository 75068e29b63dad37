set -uo pipefail
mkdir -p gpurun_out
cd /tmp; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/g33prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --matrix lj --steps 1 --warmup 0 --tiled 0 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/g33prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
grep '^{"metric"' gpurun_out/g33prof.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'],d['config']['path'],d['config']['numblkC'],d['roofline']['kernel'][:40])"
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/g33prof/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:20]:
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>5s} tot_ms {float(r["TotalDurationNs"])/1e6:9.1f} {100*float(r["TotalDurationNs"])/tot:5.1f}%')
PY
