set -e
mkdir -p gpurun_out/g6
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_tiled_full.py > gpurun_out/g6/tiled.log 2>&1 || true
tail -5 gpurun_out/g6/tiled.log
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ --ignore=tests/test_gpu_tiled_full.py > gpurun_out/g6/gpu.log 2>&1
tail -3 gpurun_out/g6/gpu.log
