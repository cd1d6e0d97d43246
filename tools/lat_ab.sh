for v in a_prev b_fold a_prev b_fold; do
  TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/variants/lib_$v.so timeout -k 10 120 python tools/bench_latency.py --methods bf16 --nq 1,8,32,256 > gpurun_out/lat_$v.json 2>&1 || exit 1
  echo "$v $(cat gpurun_out/lat_$v.json | tail -1)"
done
