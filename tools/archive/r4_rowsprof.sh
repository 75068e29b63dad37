#!/bin/bash
# per-phase clocks of the row-merge classes (libtsg_prof.so, -DTSG_ROWS_PROF): bash tools/r4_rowsprof.sh TAG bench-args
set -uo pipefail
TAG=$1; shift
mkdir -p gpurun_out
TSG_LIB_PATH=$PWD/spgemm_amd/lib/libtsg_prof.so timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --tiled 0 "$@" > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err || { tail -3 gpurun_out/${TAG}.err; exit 1; }
grep "^rows" gpurun_out/${TAG}.err | tail -3
