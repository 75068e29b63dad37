#!/bin/bash
# usage: bash tools/ks.sh <tag> [bench args]: rocprofv3 kernel stats of bench.py
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ks_$TAG -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $R/gpurun_out/ks_$TAG.log 2>&1 || exit 1
cd $R && python3 tools/kstats.py $(find gpurun_out/ks_$TAG -name "*kernel_stats.csv") 7 | head -${KS_TOP:-14}
