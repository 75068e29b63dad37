#!/bin/bash
# the drop-in tiled path (tsg_tilespgemm): its tests, then webbase and cant lines
set -uo pipefail
TAG=${1:-r4t}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tiled_full.py tests/test_gpu_parity.py > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_tests.log | head -20; exit 1; }
for mat in webbase cant; do
  timeout -k 10 300 python3 -u bench.py --matrix $mat --leg tiled --steps 5 --warmup 2 > gpurun_out/${TAG}_$mat.json 2> gpurun_out/${TAG}_$mat.err || { tail -3 gpurun_out/${TAG}_$mat.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$mat.json'));t=d['tiled'];print('$mat',t['t_kern_tiled_ms'],t['t_step1_ms'],t['t_step2_ms'],t['t_step3_ms'],t['numblkC'],t['nnzC'])"
done
