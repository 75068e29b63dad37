#!/bin/bash
# Build working-tree variants for timing experiments:
#   bash tools/var_build.sh name1 "-DFOO=1" name2 "-DFOO=0 -DBAR=2" ...
# -> spgemm_amd/lib/libtsg_<name>.so  (run them with tools/var_run.sh)
set -e
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  touch spgemm_amd/csrc/*.hip
  make -C spgemm_amd/csrc -j8 EXTRA="$2" > /dev/null
  cp spgemm_amd/lib/libtsg.so spgemm_amd/lib/libtsg_$1.so
  echo "built libtsg_$1.so ($2)"
  shift 2
done
touch spgemm_amd/csrc/*.hip
make -C spgemm_amd/csrc -j8 > /dev/null
