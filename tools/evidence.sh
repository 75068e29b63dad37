#!/bin/bash
# Evidence for every BASELINE config (through gpurun):
#   bash tools/evidence.sh TAG  -> profiles/TAG_<config>_{kernel_stats.txt,pmc.json,bench.json}
# each config: tools/profile.sh (separate --pmc FETCH_SIZE and --pmc WRITE_SIZE
# passes, then rocprofv3 --kernel-trace --stats of the same bench command with
# the CPU baseline on and the traffic read from this run's PMC summary).
# tiled_<m>: the drop-in tsg_tilespgemm path alone (bench.py --leg tiled).
# tiles_<m>: the device pipeline forced onto the staged tile pipeline
#   (TSG_PATH=tiles: step 1, step 2's bitmask symbolic, step 3's LDS accumulator).
# lj: the whole LiveJournal stand-in (90 row blocks; 3 steps).
set -uo pipefail
TAG=${1:-r4}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
run() {
  local cfg=$1; shift
  timeout -k 10 1000 bash tools/profile.sh "${TAG}_${cfg}" "$@" > "gpurun_out/${TAG}_${cfg}.log" 2>&1 || { echo "$cfg failed"; tail -5 "gpurun_out/${TAG}_${cfg}.log"; return 1; }
  python3 -c "import json;d=json.load(open('profiles/${TAG}_${cfg}_bench.json'));r=d['roofline'];c=d.get('cpu_baseline') or {};print('$cfg', d['ms_per_step'], d['value'], d['config']['path'], r.get('frac'), r.get('traffic'), r.get('traffic_all_kernels') or (r.get('pass') or {}).get('traffic_all_kernels'), c.get('value'), c.get('nnzC'))"
}
mkdir -p gpurun_out
for c in ${CONFIGS:-webbase cant mc2depi mawi ljblock tiled_webbase tiled_cant}; do
  case $c in
    webbase) run webbase --matrix webbase || exit 1 ;;
    cant) run cant --matrix cant || exit 1 ;;
    mc2depi) run mc2depi --matrix mc2depi || exit 1 ;;
    mawi) run mawi --matrix mawi || exit 1 ;;
    ljblock) run ljblock --matrix lj --row-start 1883808 --rows 1600 || exit 1 ;;
    tiled_webbase) run tiled_webbase --matrix webbase --leg tiled || exit 1 ;;
    tiled_cant) run tiled_cant --matrix cant --leg tiled || exit 1 ;;
    tiles_webbase) TSG_PATH=tiles run tiles_webbase --matrix webbase || exit 1 ;;
    tiles_cant) TSG_PATH=tiles run tiles_cant --matrix cant || exit 1 ;;
    lj) PSTEPS=2 run lj --matrix lj || exit 1 ;;
  esac
done
