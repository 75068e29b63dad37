set -e
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rows.py tests/test_gpu_values.py > gpurun_out/g12.log 2>&1 || true
tail -2 gpurun_out/g12.log
timeout -k 10 200 python3 tools/fz_time.py webbase --path=rows 2>&1 | grep webbase
TSG_LIB_PATH=$PWD/spgemm_amd/lib/libtsg_prof.so timeout -k 10 200 python3 tools/fz_time.py webbase --path=rows 2>&1 | tail -4 | head -1
bash tools/rows_prof.sh g12 webbase rows 2>&1 | grep -E "bitmap|compact"
