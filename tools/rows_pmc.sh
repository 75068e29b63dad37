#!/bin/bash
# SQ counters of the row-merge path's kernels on a stand-in (run through gpurun):
#   tools/rows_pmc.sh TAG MATRIX "COUNTERS"   -> gpurun_out/TAG/pmc (one --pmc pass, <= 8 SQ counters)
set -euo pipefail
TAG=${1:-rowspmc}; MAT=${2:-webbase}
CTRS=${3:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/pmc" -o run -- \
  python3 "$ROOT/tools/fz_time.py" "$MAT" --path=rows > "$OUT/pmc.log" 2>&1
cd "$ROOT"
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    if "k_rows" not in r["Kernel_Name"]: continue
    acc[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(r["Kernel_Name"][:60], r["Counter_Name"])] += 1
for kname, d in acc.items():
    calls = max(n[(kname, c)] for c in d)
    print(kname, {c: f"{v / calls:.4g}" for c, v in sorted(d.items())})
PY
