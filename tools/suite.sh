#!/bin/bash
# the GPU test suite + smoke (log under gpurun_out/$1_tests.log)
set -uo pipefail
TAG=${1:-r6}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -4 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_tests.log | head -20; exit 1; }
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG}_smoke.log; exit $rc
