# round-3 final evidence (tag from $1, default r3c): per-config rocprofv3 stats + PMC
# passes (raw under gpurun_out/<tag>_<cfg>, summarised locally by tools/pmc_summary.py),
# the default line (webbase + tiled leg + CPU baseline), cant tiled lines at 16/32/48/64,
# the full LiveJournal line -- every output under gpurun_out/ (merged back by gpurun)
set -uo pipefail
TAG=${1:-r3c}
mkdir -p gpurun_out
CONFIGS="webbase cant mc2depi mawi ljblock" bash tools/r3_profile.sh $TAG || exit 1
timeout -k 10 300 python3 -u bench.py > gpurun_out/${TAG}_default_bench.json 2> gpurun_out/${TAG}_default.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_default_bench.json'));print('default',d['ms_per_step'],d['value'],d['roofline']['frac'],d['roofline']['traffic']);print('tiled',d['tiled']['t_kern_tiled_ms'])"
for t in 16 32 48 64; do
  timeout -k 10 300 python3 -u bench.py --matrix cant --steps 5 --warmup 2 --tile $t --tiled 1 --no-cpu-baseline > gpurun_out/${TAG}_tiled_cant_t$t.json 2> gpurun_out/${TAG}_tiled_cant_t$t.err || { echo "cant $t failed"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_tiled_cant_t$t.json'));t=d['tiled'];print('cant tile',$t,t['t_kern_tiled_ms'],t['roofline']['frac'])"
done
timeout -k 10 900 python3 -u bench.py --matrix lj --steps 2 --warmup 1 --tiled 0 > gpurun_out/${TAG}_lj_bench.json 2> gpurun_out/${TAG}_lj.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_lj_bench.json'));print('lj full',d['ms_per_step'],d['value'],d['config'].get('row_blocks'))"
