set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tiled_full.py tests/test_gpu_cli_csv.py tests/test_gpu_step1_paths.py > gpurun_out/g39_tests.log 2>&1; rc=$?; tail -2 gpurun_out/g39_tests.log; [ $rc -eq 0 ] || exit 1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/g39prof -o run -- python3 $GRAFT_REPO_ROOT/tools/tiled_time.py webbase 3 > $GRAFT_REPO_ROOT/gpurun_out/g39prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT; grep "tile 16" gpurun_out/g39prof.log
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/g39prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "zero_empty" in r["Name"]: print(r["Name"][:40], r["Calls"], float(r["AverageNs"])/1e3)
PY
