set -uo pipefail
mkdir -p gpurun_out
for t in 16 32 48 64; do
  timeout -k 10 300 python3 -u bench.py --matrix cant --steps 5 --warmup 2 --tile $t --tiled 1 --no-cpu-baseline > gpurun_out/r3_tiled_cant_t$t.json 2> gpurun_out/r3_tiled_cant_t$t.err || { echo "cant $t failed"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r3_tiled_cant_t$t.json'));t=d['tiled'];print($t,t['t_kern_tiled_ms'],t['roofline']['frac'],t['roofline']['layout_frac'])"
done
CONFIGS="webbase cant mc2depi mawi ljblock" bash tools/r3_profile.sh r3a
