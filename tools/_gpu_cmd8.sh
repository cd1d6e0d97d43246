set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for so in two-tower-model-v2_amd/lib/variants/lib_*.so; do
    name=$(basename $so .so)
    for cfg in "768 16" "768 64" "768 256"; do
      set -- $cfg
      TWOTOWER_HIP_LIB=$PWD/$so timeout -k 10 120 python tools/bench_small_search.py --dim $1 --catalog 2000000 --nq $2 --reps 21 > gpurun_out/s_${name}_$1_$2_$rep.json 2>&1 || exit 3
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'dim', d['dim'], 'nq', d['nq'], 'wrapper', d['wrapper']['events_ms'], 'b2b', d['b2b_ms'])" gpurun_out/s_${name}_$1_$2_$rep.json $name
    done
  done
done
