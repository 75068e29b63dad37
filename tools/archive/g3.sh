set -e
bash tools/rows_prof.sh g3 webbase rows > gpurun_out/g3.txt 2>&1
