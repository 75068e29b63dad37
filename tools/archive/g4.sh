set -e
for gm in 0 1 0.75 2; do
  echo "gmul $gm"; TSG_ROWS_GMUL=$gm timeout -k 10 200 python3 tools/fz_time.py webbase --path=rows 2>&1 | grep webbase
done
TSG_ROWS_GMUL=0 bash tools/rows_prof.sh g4 webbase rows 2>&1 | grep merge
