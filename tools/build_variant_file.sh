#!/bin/bash
# A/B builds: libtsg.so with one source file replaced by a given version.
#   bash tools/build_variant_file.sh NAME FILE REPLACEMENT  -> spgemm_amd/lib/variants/libtsg_NAME.so
set -euo pipefail
NAME=$1; FILE=$2; REPL=$3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/tsgvar.XXXX)
mkdir -p "$W/spgemm_amd" "$W/include"
cp -r "$ROOT/spgemm_amd/csrc" "$W/spgemm_amd/"
cp "$ROOT/include/"*.h "$W/include/"
cp "$REPL" "$W/spgemm_amd/csrc/$FILE"
make -C "$W/spgemm_amd/csrc" -j8 ../lib/libtsg.so > "$W/build.log" 2>&1 || { tail -20 "$W/build.log"; exit 1; }
mkdir -p "$ROOT/spgemm_amd/lib/variants"
cp "$W/spgemm_amd/lib/libtsg.so" "$ROOT/spgemm_amd/lib/variants/libtsg_$NAME.so"
rm -rf "$W"
echo "built spgemm_amd/lib/variants/libtsg_$NAME.so"
