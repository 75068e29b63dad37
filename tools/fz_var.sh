#!/bin/bash
# A/B timing of the fused path on the GPU box: each argument is a set of env
# assignments (quoted), run in its own process (the library reads them once).
#   tools/fz_var.sh "" "TSG_FZ_TL=1024" ...   (matrices: $FZ_MATS, default webbase cant mc2depi)
MATS=${FZ_MATS:-webbase cant mc2depi}
for v in "$@"; do
  echo "== $v"
  env $v timeout -k 10 100 python tools/fz_time.py $MATS --path=fused 2>&1 | grep -v amdgpu.ids || exit 1
done
