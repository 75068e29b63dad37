# round-3 final evidence (tag r3b): per-config rocprofv3 stats + PMC passes, full LJ,
# default line (webbase + tiled leg + CPU baseline), cant tiled lines at 16/32/48/64
set -uo pipefail
mkdir -p gpurun_out
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3b_tiledprof -o run -- python3 $GRAFT_REPO_ROOT/tools/tiled_time.py webbase 3 > $GRAFT_REPO_ROOT/gpurun_out/r3b_tiledprof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT; tail -1 gpurun_out/r3b_tiledprof.log
cp $(ls gpurun_out/r3b_tiledprof/*/*kernel_stats.csv gpurun_out/r3b_tiledprof/*kernel_stats.csv 2>/dev/null | head -1) profiles/r3b_tiled_webbase_kernel_stats.csv
CONFIGS="webbase cant mc2depi mawi ljblock" bash tools/r3_profile.sh r3b || exit 1
timeout -k 10 300 python3 -u bench.py > profiles/r3b_default_bench.json 2> gpurun_out/r3b_default.err || exit 1
python3 -c "import json;d=json.load(open('profiles/r3b_default_bench.json'));print('default',d['ms_per_step'],d['value'],d['roofline']['frac'],d['roofline']['traffic']);print('tiled',d['tiled']['t_kern_tiled_ms']);print('cpu',d['cpu_baseline']['value'],d['cpu_baseline']['sample'][:80])"
for t in 16 32 48 64; do
  timeout -k 10 300 python3 -u bench.py --matrix cant --steps 5 --warmup 2 --tile $t --tiled 1 --no-cpu-baseline > profiles/r3b_tiled_cant_t$t.json 2> gpurun_out/r3b_tiled_cant_t$t.err || { echo "cant $t failed"; exit 1; }
  python3 -c "import json;d=json.load(open('profiles/r3b_tiled_cant_t$t.json'));t=d['tiled'];print('cant tile',$t,t['t_kern_tiled_ms'],t['roofline']['frac'])"
done
timeout -k 10 900 python3 -u bench.py --matrix lj --steps 2 --warmup 1 --tiled 0 > profiles/r3b_lj_bench.json 2> gpurun_out/r3b_lj.err || exit 1
python3 -c "import json;d=json.load(open('profiles/r3b_lj_bench.json'));print('lj full',d['ms_per_step'],d['value'],d['config']['path'],d['config'].get('row_blocks'))"
