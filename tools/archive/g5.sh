set -e
mkdir -p gpurun_out/g5
timeout -k 10 200 python3 tools/fz_time.py webbase --path=rows 2>&1 | grep webbase
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rows.py > gpurun_out/g5/tests.log 2>&1; tail -1 gpurun_out/g5/tests.log
bash tools/rows_prof.sh g5 webbase rows 2>&1 | grep -E "merge|small|bitmap"
KRE=k_rows_merge timeout -k 10 300 bash tools/sq_counters.sh g5sq --matrix webbase --tiled 0 > /dev/null 2>&1
python3 tools/sq_summary.py gpurun_out/g5sq | grep -E "merge|INSTS_VALU|WAVE_CYCLES|WAIT_ANY|WAIT_INST_ANY|INSTS_LDS |INSTS_SALU"
