#!/bin/bash
# Per-config bench lines on the GPU box (gpurun): one JSON line per BASELINE
# config into gpurun_out/$TAG/<config>.json (stderr beside it).
#   tools/r2_configs.sh r2b [webbase cant mc2depi lj mawi]
set -o pipefail
TAG=${1:-r2}
shift || true
CFGS=${@:-webbase cant mc2depi lj mawi}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
for c in $CFGS; do
  case $c in
    webbase) A=(--steps 10 --warmup 2) ;;
    lj|mawi) A=(--steps 3 --warmup 1 --cpu-budget-s 10) ;;
    *) A=(--steps 10 --warmup 2 --cpu-budget-s 10) ;;
  esac
  echo "== $c" >&2
  timeout -k 10 280 python3 "$ROOT/bench.py" --matrix "$c" "${A[@]}" > "$OUT/$c.json" 2> "$OUT/$c.err" || exit 1
  tail -c 300 "$OUT/$c.json" >&2
done
