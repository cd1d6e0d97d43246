#!/bin/bash
# On the GPU box: parity suites touched by the ring-level rules, then small/mid-batch latency
# A/B over lib/variants/lib_*.so (tools/bench_small_search.py, alternating x2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_batch.py tests/test_gpu_configs4.py tests/test_gpu_sharded_index.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_lvl.log 2>&1 || { tail -30 gpurun_out/pytest_lvl.log; exit 3; }
tail -2 gpurun_out/pytest_lvl.log
for rep in 1 2; do
  for so in two-tower-model-v2_amd/lib/variants/lib_*.so; do
    name=$(basename $so .so)
    for cfg in ${CFGS:-"768 16" "768 256" "768 1000" "384 256"}; do
      set -- $cfg
      TWOTOWER_HIP_LIB=$PWD/$so timeout -k 10 120 python tools/bench_small_search.py --dim $1 --catalog 2000000 --nq $2 --reps 21 > gpurun_out/s_${name}_$1_$2_$rep.json 2>&1 || exit 4
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'dim', d['dim'], 'nq', d['nq'], 'wrapper', d['wrapper']['events_ms'], 'b2b', d['b2b_ms'])" gpurun_out/s_${name}_$1_$2_$rep.json $name
    done
  done
done
