set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_batch.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_p.log 2>&1 || { tail -30 gpurun_out/pytest_p.log; exit 3; }
tail -2 gpurun_out/pytest_p.log
for rep in 1 2; do
  for so in two-tower-model-v2_amd/lib/variants/lib_*.so; do
    name=$(basename $so .so)
    for cfg in "768 16" "768 64" "768 256" "384 8" "384 64" "384 256"; do
      set -- $cfg
      TWOTOWER_HIP_LIB=$PWD/$so timeout -k 10 120 python tools/bench_small_search.py --dim $1 --catalog 2000000 --nq $2 --reps 21 > gpurun_out/s_${name}_$1_$2_$rep.json 2>&1 || exit 4
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'dim', d['dim'], 'nq', d['nq'], 'wrapper', d['wrapper']['events_ms'], 'b2b', d['b2b_ms'])" gpurun_out/s_${name}_$1_$2_$rep.json $name
    done
  done
done
REPS=2 BENCH_ARGS="--steps 10 --warmup 2" timeout -k 10 600 bash tools/bench_ab.sh > gpurun_out/ab.log 2>&1 || exit 5
cat gpurun_out/ab.log
