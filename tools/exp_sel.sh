export TMPDIR=/tmp
for v in ${SELV:-stop1 stop2}; do
  rm -rf gpurun_out/sel_$v
  TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/variants/lib_$v.so timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/sel_$v -o run --output-format csv -- python tools/bench_latency.py --methods bf16 --nq 1 > gpurun_out/sel_$v.log 2>&1 || exit 1
done
rm -rf gpurun_out/sel_base
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/sel_base -o run --output-format csv -- python tools/bench_latency.py --methods bf16 --nq 1 > gpurun_out/sel_base.log 2>&1 || exit 1
grep catalog gpurun_out/sel_base.log
