#!/bin/bash
# SQ / LDS counters of the row-merge kernels on webbase (round 4 design input).
set -uo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
KRE="k_rows" timeout -k 10 400 bash tools/sq_counters.sh r4_sq --tiled 0 > gpurun_out/r4_sq.log 2>&1 || { echo "sq failed"; tail -20 gpurun_out/r4_sq.log; exit 1; }
python3 tools/sq_summary.py gpurun_out/r4_sq > gpurun_out/r4_sq_summary.txt
cat gpurun_out/r4_sq_summary.txt
