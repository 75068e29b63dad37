#!/bin/bash
# A/B builds: libtsg.so from the sources at a git revision (default HEAD), for
# TSG_LIB_PATH runs against the working tree's build.
#   bash tools/build_variant_rev.sh NAME [REV]  -> spgemm_amd/lib/variants/libtsg_NAME.so
set -euo pipefail
NAME=$1; REV=${2:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/tsgrev.XXXX)
git -C "$ROOT" archive "$REV" spgemm_amd/csrc include | tar -x -C "$W"
make -C "$W/spgemm_amd/csrc" -j8 ../lib/libtsg.so > "$W/build.log" 2>&1 || { tail -20 "$W/build.log"; exit 1; }
mkdir -p "$ROOT/spgemm_amd/lib/variants"
cp "$W/spgemm_amd/lib/libtsg.so" "$ROOT/spgemm_amd/lib/variants/libtsg_$NAME.so"
rm -rf "$W"
echo "built spgemm_amd/lib/variants/libtsg_$NAME.so"
