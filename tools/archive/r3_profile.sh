#!/bin/bash
# Round-3 evidence for every BASELINE config (through gpurun):
#   bash tools/r3_profile.sh TAG  -> profiles/TAG_<config>_{kernel_stats.txt,pmc.json,bench.json}
# each config: tools/profile.sh (rocprofv3 --kernel-trace --stats, then separate
# --pmc FETCH_SIZE and --pmc WRITE_SIZE passes) of the same bench command.
set -uo pipefail
TAG=${1:-r3}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
run() {
  local cfg=$1; shift
  bash tools/profile.sh "${TAG}_${cfg}" "$@" > "gpurun_out/${TAG}_${cfg}.log" 2>&1 || { echo "$cfg failed"; return 1; }
  python3 -c "import json;d=json.load(open('profiles/${TAG}_${cfg}_bench.json'));print('$cfg', d['ms_per_step'], d['value'], d['config']['path'], d['roofline']['frac'], d['roofline']['traffic'])"
}
mkdir -p gpurun_out
for c in ${CONFIGS:-webbase cant mc2depi mawi ljblock}; do
  case $c in
    webbase) run webbase --matrix webbase || exit 1 ;;
    cant) run cant --matrix cant || exit 1 ;;
    mc2depi) run mc2depi --matrix mc2depi || exit 1 ;;
    mawi) run mawi --matrix mawi || exit 1 ;;
    ljblock) run ljblock --matrix lj --row-start 1883808 --rows 1600 || exit 1 ;;
  esac
done
