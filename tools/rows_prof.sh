#!/bin/bash
# per-kernel times of one path on a stand-in (run through gpurun):
#   tools/rows_prof.sh TAG MATRIX PATH  -> gpurun_out/TAG/stats (rocprofv3 --kernel-trace --stats)
set -euo pipefail
TAG=${1:-rows}; MAT=${2:-webbase}; P=${3:-rows}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TSG_PATH=$P
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
  python3 "$ROOT/bench.py" --matrix "$MAT" --steps 5 --warmup 2 --no-cpu-baseline --tiled 0 > "$OUT/stats.log" 2>&1
cd "$ROOT"
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/stats/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:9.1f} tot_ms {float(r["TotalDurationNs"])/1e6:8.2f}')
PY
