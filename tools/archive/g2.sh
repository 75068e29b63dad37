set -e
mkdir -p gpurun_out/g2
timeout -k 10 200 python3 tools/fz_time.py webbase --path=rows > gpurun_out/g2/base.log 2>&1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rows.py tests/test_gpu_values.py > gpurun_out/g2/tests.log 2>&1
TSG_LIB_PATH=$PWD/spgemm_amd/lib/libtsg_prof.so timeout -k 10 200 python3 tools/fz_time.py webbase --path=rows > gpurun_out/g2/prof.log 2>&1
