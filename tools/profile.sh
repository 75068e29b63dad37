#!/bin/bash
# Profile of one bench command on the GPU box (run through gpurun):
#   1) rocprofv3 --pmc FETCH_SIZE  (own pass)          -> gpurun_out/$TAG/pmc_fetch
#   2) rocprofv3 --pmc WRITE_SIZE  (own pass)          -> gpurun_out/$TAG/pmc_write
#   3) summarise the counters                          -> profiles/$TAG_pmc.json
#   4) rocprofv3 --kernel-trace --stats, CPU baseline on, the line's traffic read
#      from step 3's summary (same build, same round)  -> gpurun_out/$TAG/stats
#   5) summarise                                       -> profiles/$TAG_{kernel_stats.*,pmc.json,bench.json}
# Counters are never combined with sys/runtime/API traces (pool rule).
set -euo pipefail
TAG=${1:-r1}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
PS=${PSTEPS:-5}
BENCH_PMC=(python3 "$ROOT/bench.py" --steps $PS --warmup 2 --no-cpu-baseline --tiled 0 "$@")
BENCH_STATS=(python3 "$ROOT/bench.py" --steps $PS --warmup 2 --tiled 0 --pmc-from "$ROOT/profiles/${TAG}_pmc.json" "$@")
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- "${BENCH_PMC[@]}" \
  > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- "${BENCH_PMC[@]}" \
  > "$OUT/pmc_write.log" 2>&1
cd "$ROOT"
python3 tools/pmc_summary.py "$OUT" "$TAG"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- "${BENCH_STATS[@]}" \
  > "$OUT/stats.log" 2>&1
cd "$ROOT"
python3 tools/pmc_summary.py "$OUT" "$TAG"
