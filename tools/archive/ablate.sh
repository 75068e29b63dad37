#!/bin/bash
# Diagnostics: time the pipeline with parts skipped (TSG_ABLATE bitmask; results
# invalid except for 0 and 16).  4 = no step-3 values, 8 = no CSR writes,
# 16 = tile-payload value pass instead of element streaming.
for a in 0 4 8 16; do
  echo "ablate=$a $(TSG_ABLATE=$a timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stage_ms"])')"
done
