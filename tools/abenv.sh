#!/bin/bash
# A/B of an environment setting: bash tools/abenv.sh TAG "VAR=VALUE" bench-args
set -uo pipefail
TAG=$1; ENVSET=$2; shift 2
mkdir -p gpurun_out
for rep in 1 2; do
  for v in base env; do
    if [ $v = env ]; then E="$ENVSET"; else E="TSG_AB_BASE=1"; fi
    env $E timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --tiled 0 "$@" > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err || { echo "$v failed"; tail -3 gpurun_out/${TAG}_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$v.json'));t=d.get('tiled') or {};print('$v', d['ms_per_step'], (d.get('stage_ms') or {}).get('t_step3_kernel_ms'), t.get('t_step1_ms'), t.get('t_step2_ms'), t.get('t_step3_ms'))"
  done
done
