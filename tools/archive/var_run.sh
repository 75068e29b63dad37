#!/bin/bash
# On the GPU box: time the variants built by tools/var_build.sh, interleaved.
# usage: bash tools/var_run.sh "name1 name2 ..." [bench args...]
NAMES=$1; shift
for rep in 1 2; do
  for L in $NAMES; do
    export TSG_LIB_PATH=$PWD/spgemm_amd/lib/libtsg_$L.so
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/var_$L.log 2>&1 || exit 1
    echo $L $(grep -o '"ms_per_step": [0-9.]*\|"t_step[123]_ms": [0-9.]*' gpurun_out/var_$L.log)
  done
done
