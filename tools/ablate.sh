#!/bin/bash
# Diagnostics: time step 3 with parts skipped (TSG_ABLATE bitmask, results invalid).
for a in 0 1 2 4 8 14 15; do
  echo "ablate=$a $(TSG_ABLATE=$a python bench.py --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["stage_ms"])')"
done
