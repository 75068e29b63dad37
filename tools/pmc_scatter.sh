#!/bin/bash
# Counters of the windowed-row kernels on the heaviest LiveJournal block, one
# rocprofv3 --pmc pass per counter group (never with traces):
#   bash tools/pmc_scatter.sh TAG  -> gpurun_out/TAG/<group>/run_counter_collection.csv
set -uo pipefail
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
B=(python3 "$ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --tiled 0 --matrix lj --row-start 1883808 --rows 1600)
cd /tmp
export TMPDIR=/tmp
i=0
for grp in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "TA_BUSY_avr TA_TA_BUSY_sum"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/g$i" -o run -- "${B[@]}" > "$OUT/g$i.log" 2>&1 || echo "group $i failed: $grp"
done
cd "$ROOT"
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for f in sorted(glob.glob(out + "/g*/run_counter_collection.csv")):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_rows_w" in k:
            agg[(k.split("(")[0], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, c), v in sorted(agg.items()):
        print(f.split("/")[-2], k, c, v)
PY
