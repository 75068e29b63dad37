set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rows.py > gpurun_out/g25_rows.log 2>&1; rc=$?; tail -5 gpurun_out/g25_rows.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_dist.py > gpurun_out/g25_cfg.log 2>&1; rc=$?; tail -5 gpurun_out/g25_cfg.log; [ $rc -eq 0 ] || exit 1
LJ="--matrix lj --row-start 1883808 --rows 1600 --steps 3 --warmup 1 --no-cpu-baseline --tiled 0"
timeout -k 10 300 python3 bench.py $LJ > gpurun_out/g25_lj.json 2>gpurun_out/g25_lj.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/g25_lj.json'));print('lj block',d['ms_per_step'],d['value'],d['config']['path'])"
timeout -k 10 300 python3 bench.py --matrix mawi --steps 3 --warmup 1 --no-cpu-baseline --tiled 0 > gpurun_out/g25_mawi.json 2>gpurun_out/g25_mawi.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/g25_mawi.json'));print('mawi',d['ms_per_step'],d['value'],d['config']['path'])"
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/g25prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py $LJ > $GRAFT_REPO_ROOT/gpurun_out/g25prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/g25prof/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:9.1f}')
PY
