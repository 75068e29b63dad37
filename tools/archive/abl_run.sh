#!/bin/bash
# On the GPU box: A/B one build under TSG_ABLATE settings, interleaved.
# usage: bash tools/abl_run.sh "0 4096" [bench args...]
VALS=$1; shift
for rep in 1 2; do
  for a in $VALS; do
    TSG_ABLATE=$a timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/abl_$a.log 2>&1 || exit 1
    echo abl=$a $(grep -o '"ms_per_step": [0-9.]*\|"t_step[123]_ms": [0-9.]*\|"t_step3_kernel_ms": [0-9.]*' gpurun_out/abl_$a.log)
  done
done
