set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rows.py tests/test_gpu_values.py tests/test_gpu_parity.py > gpurun_out/g23_tests.log 2>&1; rc=$?; tail -3 gpurun_out/g23_tests.log; [ $rc -eq 0 ] || exit 1
for v in 1 0 1 0; do echo "staged=$v"; TSG_ROWS_STAGED=$v timeout -k 10 200 python3 tools/fz_time.py webbase mc2depi --path=rows 2>&1 | grep -v amdgpu.ids || exit 1; done
timeout -k 10 300 bash tools/rows_prof.sh g23 webbase rows 2>&1 | tail -30
