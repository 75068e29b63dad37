#!/bin/bash
# SQ / LDS / L2 counters for the step kernels (separate --pmc passes, no traces).
# usage (through gpurun): bash tools/sq_counters.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-sq}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
BENCH=(python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline "$@")
cd /tmp
export TMPDIR=/tmp
n=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU" \
           "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  n=$((n+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "${KRE:-k_step|k_eseg|k_esplit}" --output-format csv \
    -d "$OUT/p$n" -o run -- "${BENCH[@]}" > "$OUT/p$n.log" 2>&1
done
