set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rows.py > gpurun_out/g18.log 2>&1; rc=$?; tail -3 gpurun_out/g18.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 tools/fz_time.py webbase --path=rows 2>&1 | tail -1 || exit 1
TSG_LIB_PATH=$PWD/spgemm_amd/lib/libtsg_prof.so timeout -k 10 200 python3 tools/fz_time.py webbase --path=rows 2>&1 | tail -4
