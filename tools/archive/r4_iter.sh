#!/bin/bash
# round 4 iteration: rows + tiled tests, then the webbase / mc2depi device lines and the webbase / cant tiled lines
set -uo pipefail
TAG=${1:-r4i}
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rows.py tests/test_gpu_tiled_full.py tests/test_gpu_parity.py > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_tests.log | head -20; exit 1; }
for mat in webbase mc2depi; do
  timeout -k 10 300 python3 -u bench.py --matrix $mat --no-cpu-baseline --tiled 0 > gpurun_out/${TAG}_$mat.json 2> gpurun_out/${TAG}_$mat.err || { tail -3 gpurun_out/${TAG}_$mat.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$mat.json'));print('$mat',d['ms_per_step'],d['value'],d['stage_ms']['t_step1_ms'],d['stage_ms']['t_step3_ms'],d['stage_ms']['t_step3_kernel_ms'])"
done
for mat in webbase cant; do
  timeout -k 10 300 python3 -u bench.py --matrix $mat --leg tiled --steps 5 --warmup 2 > gpurun_out/${TAG}_t$mat.json 2> gpurun_out/${TAG}_t$mat.err || { tail -3 gpurun_out/${TAG}_t$mat.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_t$mat.json'));t=d['tiled'];print('tiled $mat',t['t_kern_tiled_ms'],t['t_step1_ms'],t['t_step2_ms'],t['t_step3_ms'])"
done
