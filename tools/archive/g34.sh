set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rows.py > gpurun_out/g34_rows.log 2>&1; rc=$?; tail -2 gpurun_out/g34_rows.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 bash tools/rows_prof.sh g34 webbase rows 2>&1 | grep -E "compact|bitmap|e2e" || exit 1
grep -E "e2e" gpurun_out/g34/stats.log | head -2
bash tools/g33.sh
