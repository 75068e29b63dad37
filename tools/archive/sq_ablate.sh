#!/bin/bash
# Instruction counts of the step kernels under TSG_ABLATE settings (one --pmc
# pass each, no traces): which phase issues the VALU/SALU/LDS instructions.
# usage (through gpurun): bash tools/sq_ablate.sh <tag> "0 4 8" [bench args...]
set -uo pipefail
TAG=${1:-sqa}; ABL=${2:-"0 4 8"}; shift 2 || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
for a in $ABL; do
  TSG_ABLATE=$a timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES \
    --kernel-include-regex "k_step" --output-format csv -d "$OUT/a$a" -o run -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline "$@" > "$OUT/a$a.log" 2>&1 || exit 1
done
