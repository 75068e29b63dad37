set -e
mkdir -p gpurun_out/g10
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rows.py tests/test_gpu_values.py tests/test_gpu_parity.py -k "rows or mawi or values or full_size" > gpurun_out/g10/tests.log 2>&1 || true
tail -3 gpurun_out/g10/tests.log
for P in default rows; do
  if [ $P = rows ]; then export TSG_PATH=rows; else unset TSG_PATH; fi
  timeout -k 10 300 python3 bench.py --matrix mawi --steps 3 --warmup 1 --no-cpu-baseline --tiled 0 > gpurun_out/g10/mawi_$P.json 2> gpurun_out/g10/mawi_$P.err
  python3 -c "import json;d=json.load(open('gpurun_out/g10/mawi_$P.json'));print('mawi $P', d['ms_per_step'], d['value'], d['config']['path'], d['stage_ms'])"
done
