set -e
mkdir -p gpurun_out/g7
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rows.py tests/test_gpu_values.py > gpurun_out/g7/tests.log 2>&1; tail -1 gpurun_out/g7/tests.log
timeout -k 10 200 python3 tools/fz_time.py webbase --path=rows 2>&1 | grep webbase
TSG_LIB_PATH=$PWD/spgemm_amd/lib/libtsg_prof.so timeout -k 10 200 python3 tools/fz_time.py webbase --path=rows 2>&1 | tail -4
bash tools/rows_prof.sh g7 webbase rows 2>&1 | grep -E "hwin|merge|small|compact"
