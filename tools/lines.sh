#!/bin/bash
# Plain bench lines (no profiler) for every BASELINE config, through gpurun:
#   bash tools/lines.sh TAG [configs...]  -> gpurun_out/TAG_<config>.json (one JSON line each)
set -uo pipefail
TAG=$1; shift
mkdir -p gpurun_out
for c in ${@:-default cant mc2depi mawi ljblock lj}; do
  case $c in
    default) args=() ;;
    ljblock) args=(--matrix lj --row-start 1883808 --rows 1600) ;;
    lj) args=(--matrix lj --steps 3 --warmup 1) ;;
    mawi) args=(--matrix mawi --steps 5) ;;
    *) args=(--matrix $c) ;;
  esac
  timeout -k 10 900 python3 -u bench.py "${args[@]}" > gpurun_out/${TAG}_$c.json 2> gpurun_out/${TAG}_$c.err \
    || { echo "$c failed"; tail -5 gpurun_out/${TAG}_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$c.json'));t=d.get('tiled') or {};c=d.get('cpu_baseline') or {};print('$c', d['ms_per_step'], d['value'], d['roofline']['frac'], (d['roofline'].get('pass') or {}).get('frac'), t.get('t_kern_tiled_ms'), c.get('value'))"
done
