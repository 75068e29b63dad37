set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rows.py -k direct > gpurun_out/g24_tests.log 2>&1; rc=$?; tail -3 gpurun_out/g24_tests.log; [ $rc -eq 0 ] || exit 1
LJ="--matrix lj --row-start 1883808 --rows 1600 --steps 3 --warmup 1 --no-cpu-baseline --tiled 0"
timeout -k 10 300 python3 bench.py $LJ > gpurun_out/g24_lj_default.json 2>gpurun_out/g24_lj_default.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/g24_lj_default.json'));print('lj default',d['ms_per_step'],d['config']['path'])"
export TSG_PATH=rows
timeout -k 10 300 python3 bench.py $LJ > gpurun_out/g24_lj_rows.json 2>gpurun_out/g24_lj_rows.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/g24_lj_rows.json'));print('lj rows',d['ms_per_step'],d['config']['path'])"
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/g24prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py $LJ > $GRAFT_REPO_ROOT/gpurun_out/g24prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT; unset TSG_PATH
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/g24prof/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:9.1f}')
PY
timeout -k 10 300 python3 bench.py > gpurun_out/g24_default.json 2>gpurun_out/g24_default.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/g24_default.json'));print('default',d['ms_per_step'],d['value'],d['roofline']['frac']);print('tiled',d['tiled'])"
