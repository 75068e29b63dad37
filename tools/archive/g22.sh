set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/g22_tests.log 2>&1; rc=$?; tail -3 gpurun_out/g22_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/g22_bench.log 2>gpurun_out/g22_bench.err; rc=$?; tail -c 3000 gpurun_out/g22_bench.log; exit $rc
