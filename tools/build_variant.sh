#!/bin/bash
# A/B builds: libtsg.so with one source edit, for TSG_LIB_PATH runs on the GPU box.
#   bash tools/build_variant.sh NAME FILE SED_EXPR  -> spgemm_amd/lib/variants/libtsg_NAME.so
set -euo pipefail
NAME=$1; FILE=$2; EXPR=$3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/tsgvar.XXXX)
mkdir -p "$W/spgemm_amd" "$W/include"
cp -r "$ROOT/spgemm_amd/csrc" "$W/spgemm_amd/"
cp "$ROOT/include/"*.h "$W/include/"
changed=0
for f in $FILE; do  # (one or more files, space-separated)
  sed -i "$EXPR" "$W/spgemm_amd/csrc/$f"
  cmp -s "$ROOT/spgemm_amd/csrc/$f" "$W/spgemm_amd/csrc/$f" || changed=1
done
[ $changed = 1 ] || { echo "sed changed nothing"; exit 1; }
make -C "$W/spgemm_amd/csrc" -j8 ../lib/libtsg.so > "$W/build.log" 2>&1 || { tail -20 "$W/build.log"; exit 1; }
mkdir -p "$ROOT/spgemm_amd/lib/variants"
cp "$W/spgemm_amd/lib/libtsg.so" "$ROOT/spgemm_amd/lib/variants/libtsg_$NAME.so"
rm -rf "$W"
echo "built spgemm_amd/lib/variants/libtsg_$NAME.so"
