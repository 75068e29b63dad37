set -e
mkdir -p gpurun_out/g1
timeout -k 10 200 python3 tools/fz_time.py webbase --path=rows > gpurun_out/g1/base.log 2>&1
TSG_LIB_PATH=$PWD/spgemm_amd/lib/libtsg_prof.so timeout -k 10 200 python3 tools/fz_time.py webbase --path=rows > gpurun_out/g1/prof.log 2>&1
KRE=k_rows timeout -k 10 600 bash tools/sq_counters.sh g1sq --matrix webbase --tiled 0 > gpurun_out/g1/sq.log 2>&1
