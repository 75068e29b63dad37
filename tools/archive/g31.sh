set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rows.py tests/test_gpu_configs.py tests/test_gpu_dist.py > gpurun_out/g31_rows.log 2>&1; rc=$?; tail -3 gpurun_out/g31_rows.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 tools/w_ab.py 6 2>&1 | grep -v amdgpu.ids || exit 1
