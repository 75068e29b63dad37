#!/bin/bash
# Round profile of the default bench workload on the GPU box (run through gpurun):
#   1) rocprofv3 --kernel-trace --stats            -> gpurun_out/$TAG/stats
#   2) rocprofv3 --pmc FETCH_SIZE  (own pass)       -> gpurun_out/$TAG/pmc_fetch
#   3) rocprofv3 --pmc WRITE_SIZE  (own pass)       -> gpurun_out/$TAG/pmc_write
# then summarises them into profiles/$TAG_* (tools/pmc_summary.py).
# Counters are never combined with sys/runtime/API traces (pool rule).
set -euo pipefail
TAG=${1:-r1}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
BENCH=(python3 "$ROOT/bench.py" --steps ${PSTEPS:-5} --warmup 2 --no-cpu-baseline --tiled 0 "$@")
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- "${BENCH[@]}" \
  > "$OUT/stats.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- "${BENCH[@]}" \
  > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- "${BENCH[@]}" \
  > "$OUT/pmc_write.log" 2>&1
cd "$ROOT"
python3 tools/pmc_summary.py "$OUT" "$TAG" 7
