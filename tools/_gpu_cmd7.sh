set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for so in two-tower-model-v2_amd/lib/variants/lib_*.so; do
    name=$(basename $so .so)
    for nq in 16 256; do
      TWOTOWER_HIP_LIB=$PWD/$so timeout -k 10 120 python tools/bench_small_search.py --dim 768 --catalog 2000000 --nq $nq --reps 21 > gpurun_out/s_${name}_${nq}_$rep.json 2>&1 || exit 3
      echo "$name nq $nq $(tail -1 gpurun_out/s_${name}_${nq}_$rep.json | cut -c1-200)"
    done
  done
done
REPS=2 BENCH_ARGS="--steps 3 --warmup 1 --dim 768 --catalog 10000000" timeout -k 10 900 bash tools/bench_ab.sh > gpurun_out/ab.log 2>&1 || exit 4
cat gpurun_out/ab.log
