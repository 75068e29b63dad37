#!/bin/bash
# round 4: first GPU check of the ordered-batch row-merge route
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rows.py > gpurun_out/r4_ob1_rows.log 2>&1; rc=$?
tail -15 gpurun_out/r4_ob1_rows.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --tiled 0 > gpurun_out/r4_ob1_web.json 2> gpurun_out/r4_ob1_web.err || { tail -5 gpurun_out/r4_ob1_web.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4_ob1_web.json'));print('webbase',d['ms_per_step'],d['value'],d['roofline']['frac'],d['stage_ms'])"
timeout -k 10 200 python3 -u bench.py --matrix mc2depi --no-cpu-baseline --tiled 0 > gpurun_out/r4_ob1_mc.json 2> gpurun_out/r4_ob1_mc.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r4_ob1_mc.json'));print('mc2depi',d['ms_per_step'],d['value'],d['stage_ms'])"
