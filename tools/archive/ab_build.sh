#!/bin/bash
# Build the committed HEAD's libtsg.so as spgemm_amd/lib/libtsg_base.so next to
# the working tree's build (A/B timing with TSG_LIB_PATH; see tools/ab_run.sh).
set -e
cd "$(dirname "$0")/.."
git stash -q
make -C spgemm_amd/csrc -j8 > /dev/null
cp spgemm_amd/lib/libtsg.so spgemm_amd/lib/libtsg_base.so
git stash pop -q
touch spgemm_amd/csrc/*.hip spgemm_amd/csrc/*.cpp
make -C spgemm_amd/csrc -j8 > /dev/null
echo "built libtsg_base.so (HEAD) and libtsg.so (working tree)"
