#!/bin/bash
# On the GPU box: alternate HEAD (base) and working-tree (cur) builds.
# usage: bash tools/ab_run.sh [bench args...]
for L in base cur base cur; do
  if [ $L = base ]; then export TSG_LIB_PATH=$PWD/spgemm_amd/lib/libtsg_base.so; else unset TSG_LIB_PATH; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/ab_$L.log 2>&1 || exit 1
  echo $L $(grep -o '"ms_per_step": [0-9.]*\|"t_csr2tile_ms": [0-9.]*\|"t_step[123]_ms": [0-9.]*' gpurun_out/ab_$L.log)
done
