set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rows.py tests/test_gpu_configs.py > gpurun_out/g35_rows.log 2>&1; rc=$?; tail -2 gpurun_out/g35_rows.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 tools/w_ab.py 6 2>&1 | grep -v amdgpu.ids || exit 1
cd /tmp; export TMPDIR=/tmp
LJ="--matrix lj --row-start 1883808 --rows 1600 --steps 5 --warmup 1 --no-cpu-baseline --tiled 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/g35prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py $LJ > $GRAFT_REPO_ROOT/gpurun_out/g35prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/g35prof/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:6]:
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:9.1f}')
PY
