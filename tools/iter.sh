#!/bin/bash
# One iteration on the GPU box (through gpurun): tests named in $TESTS (pytest
# -k expression in $K), then A/B bench lines and a kernel-stats profile.
#   TESTS="tests/test_gpu_rows.py ..." K="expr" AB="cant:oldband" ENVAB="webbase:TSG_ROWS_DIRECT=0" \
#   PROF="webbase" bash tools/iter.sh TAG
set -uo pipefail
TAG=$1
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS ${K:+-k "$K"} \
    > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
  tail -3 gpurun_out/${TAG}_tests.log
  [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_tests.log | head -20; exit 1; }
fi
for ab in ${AB:-}; do  # matrix:variant (spgemm_amd/lib/variants/libtsg_<variant>.so)
  bash tools/ab.sh ${TAG}_${ab%%:*} "${ab#*:}" --matrix ${ab%%:*} || exit 1
done
for ab in ${TAB:-}; do  # matrix:variant, the tiled drop-in leg (tsg_tilespgemm)
  bash tools/ab.sh ${TAG}_tiled_${ab%%:*} "${ab#*:}" --matrix ${ab%%:*} --leg tiled --steps 5 || exit 1
done
for ab in ${ENVAB:-}; do  # matrix:VAR=VALUE
  bash tools/abenv.sh ${TAG}_${ab%%:*} "${ab#*:}" --matrix ${ab%%:*} || exit 1
done
for m in ${PROF:-}; do  # kernel trace + stats of one bench command
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OLDPWD/gpurun_out/${TAG}_prof_$m" -o run -- python3 "$OLDPWD/bench.py" --matrix $m --steps 5 --warmup 2 \
      --no-cpu-baseline --tiled 0 ) > gpurun_out/${TAG}_prof_$m.log 2>&1 || { echo "prof $m failed"; tail -5 gpurun_out/${TAG}_prof_$m.log; exit 1; }
  f=$(find gpurun_out/${TAG}_prof_$m -name "*kernel_stats.csv" | sort | sed -n 1p)
  python3 tools/kstats.py "$f" 7 > gpurun_out/${TAG}_prof_$m.txt && sed -n 1,26p gpurun_out/${TAG}_prof_$m.txt
done
