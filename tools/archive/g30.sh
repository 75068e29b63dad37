set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/g30_tests.log 2>&1; rc=$?; tail -3 gpurun_out/g30_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g30_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/g30_smoke.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/g30_bench.json 2>gpurun_out/g30_bench.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/g30_bench.json'));print('default',d['ms_per_step'],d['value'],d['roofline']['frac'])"
