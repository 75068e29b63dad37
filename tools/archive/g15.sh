for t in 16 32 48 64; do timeout -k 10 300 python3 tools/tiled_time.py cant 3 $t 2>&1 | grep t_tile; done
for t in 32 64; do timeout -k 10 300 python3 tools/tiled_time.py webbase 2 $t 2>&1 | grep t_tile; done
