#!/bin/bash
# kernel stats of one bench command (round 4 iteration): bash tools/r4_ks.sh TAG [bench args]
set -uo pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --tiled 0 "$@" > "$OUT/stats.log" 2>&1 || { tail -5 "$OUT/stats.log"; exit 1; }
cd "$ROOT"
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/stats/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:22]:
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:9.1f}')
PY
grep '^{"metric"' "$OUT/stats.log" | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'],d.get('stage_ms') or {k: v for k, v in (d.get('tiled') or {}).items() if k.startswith('t_')})"
