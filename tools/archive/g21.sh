set -uo pipefail
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_dist.py > gpurun_out/g21.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/g21.log | tail -12; exit $rc
