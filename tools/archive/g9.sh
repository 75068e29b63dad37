set -e
mkdir -p gpurun_out/g9
for P in default rows; do
  if [ $P = rows ]; then export TSG_PATH=rows; else unset TSG_PATH; fi
  timeout -k 10 300 python3 bench.py --matrix mawi --steps 3 --warmup 1 --no-cpu-baseline --tiled 0 > gpurun_out/g9/mawi_$P.json 2> gpurun_out/g9/mawi_$P.err
  python3 -c "import json;d=json.load(open('gpurun_out/g9/mawi_$P.json'));print('mawi $P', d['ms_per_step'], d['value'], d['config']['path'])"
  timeout -k 10 400 python3 bench.py --matrix lj --steps 1 --warmup 1 --no-cpu-baseline --tiled 0 > gpurun_out/g9/lj_$P.json 2> gpurun_out/g9/lj_$P.err
  python3 -c "import json;d=json.load(open('gpurun_out/g9/lj_$P.json'));print('lj $P', d['ms_per_step'], d['value'], d['config']['path'])"
done
