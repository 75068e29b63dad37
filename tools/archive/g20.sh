set -uo pipefail
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rows.py > gpurun_out/g20.log 2>&1; rc=$?; tail -3 gpurun_out/g20.log; [ $rc -eq 0 ] || exit 1
for k in 1 2 3 4; do echo "segs $k"; TSG_ROWS_SEGS=$k timeout -k 10 200 python3 tools/fz_time.py webbase mc2depi --path=rows 2>&1 | tail -2 || exit 1; done
