for rep in 1 2 3; do
for L in base v1 cur; do
  if [ $L = cur ]; then unset TSG_LIB_PATH; else export TSG_LIB_PATH=$PWD/spgemm_amd/lib/libtsg_$L.so; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --tiled 0 > gpurun_out/abv_$L.log 2>&1 || exit 1
  echo $L $(grep -o '"ms_per_step": [0-9.]*\|"t_step3_ms": [0-9.]*' gpurun_out/abv_$L.log)
done
done
