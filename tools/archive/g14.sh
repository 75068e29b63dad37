set -e
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_rows.py tests/test_gpu_fused.py tests/test_gpu_parity.py > gpurun_out/g14.log 2>&1 || true
tail -3 gpurun_out/g14.log
timeout -k 10 300 python3 bench.py --matrix mc2depi --steps 10 --no-cpu-baseline --tiled 0 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.readline());print('mc2depi', d['ms_per_step'], d['value'], d['config']['path'])"
