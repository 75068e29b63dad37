#!/bin/bash
# Kernel stats of one bench command per library variant (main + variants):
#   bash tools/prof_variants.sh TAG "variant ..." bench args...
# -> gpurun_out/TAG_<variant>.txt (tools/kstats.py of rocprofv3 --kernel-trace --stats)
set -uo pipefail
TAG=$1; VARS=$2; shift 2
ROOT=$(pwd)
mkdir -p gpurun_out
for v in main $VARS; do
  if [ "$v" = main ]; then unset TSG_LIB_PATH; else export TSG_LIB_PATH=$ROOT/spgemm_amd/lib/variants/libtsg_$v.so; fi
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$ROOT/gpurun_out/${TAG}_$v" -o run -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 \
      --no-cpu-baseline --tiled 0 "$@" ) > gpurun_out/${TAG}_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/${TAG}_$v.log; exit 1; }
  f=$(find gpurun_out/${TAG}_$v -name "*kernel_stats.csv" | sort | sed -n 1p)
  python3 tools/kstats.py "$f" 5 > gpurun_out/${TAG}_$v.txt
  echo "== $v"; sed -n 1,9p gpurun_out/${TAG}_$v.txt
done
