set -e
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/g13.log 2>&1 || true
tail -4 gpurun_out/g13.log
timeout -k 10 200 python3 tools/fz_time.py webbase mc2depi cant --path=rows,fused,band 2>&1 | grep -v amdgpu.ids
