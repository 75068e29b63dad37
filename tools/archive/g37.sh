set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_rows.py tests/test_gpu_api_threads.py > gpurun_out/g37_tests.log 2>&1; rc=$?; tail -2 gpurun_out/g37_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/g32.sh r3e
