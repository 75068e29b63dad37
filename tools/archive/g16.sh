timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "other_tile or dense_acc or stages or cli" > gpurun_out/g16.log 2>&1; tail -2 gpurun_out/g16.log
for t in 16 32 48 64; do timeout -k 10 300 python3 tools/tiled_time.py cant 3 $t 2>&1 | grep t_tile; done
for t in 32 64; do timeout -k 10 300 python3 tools/tiled_time.py webbase 2 $t 2>&1 | grep t_tile; done
