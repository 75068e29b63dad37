set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r3d_gputest.log 2>&1; rc=$?; tail -2 gpurun_out/r3d_gputest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3d_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r3d_smoke.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python3 -u bench.py --matrix lj --steps 2 --warmup 1 --tiled 0 > gpurun_out/r3d_lj_bench.json 2> gpurun_out/r3d_lj.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r3d_lj_bench.json'));print('lj full',d['ms_per_step'],d['value'],d['config']['path'],d['config'].get('row_blocks'))"
timeout -k 10 300 python3 -u bench.py > gpurun_out/r3d_default_bench.json 2> gpurun_out/r3d_default.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r3d_default_bench.json'));print('default',d['ms_per_step'],d['value'],d['roofline']['frac'])"
timeout -k 10 300 python3 -u bench.py --matrix mawi --steps 5 --warmup 1 --tiled 0 --no-cpu-baseline > gpurun_out/r3d_mawi_bench.json 2> gpurun_out/r3d_mawi.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r3d_mawi_bench.json'));print('mawi',d['ms_per_step'],d['value'],d['roofline']['frac'])"
