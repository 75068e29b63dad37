set -e
mkdir -p gpurun_out/g8
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rows.py > gpurun_out/g8/tests.log 2>&1 || true
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/g8/tests.log | tail -30
timeout -k 10 200 python3 tools/fz_time.py webbase --path=rows 2>&1 | grep webbase
