#!/bin/bash
# On the GPU box: filter/scan parity tests + headline bench (Mode B only) for A/B env settings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded_index.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/filter_tests.log 2>&1 || { tail -30 gpurun_out/filter_tests.log; exit 1; }
tail -1 gpurun_out/filter_tests.log
for envs in ${AB:-"X=1"}; do
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --mode-a-buyers 0 --steps 5 --warmup 2 > gpurun_out/bench_ab.log 2>&1 || { tail -5 gpurun_out/bench_ab.log; exit 1; }
  echo "$envs $(grep -o '"value": [0-9.]*' gpurun_out/bench_ab.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/bench_ab.log) $(grep -o '"search_ms": [0-9.]*' gpurun_out/bench_ab.log) $(grep -o '"fallback_queries_last_step": [0-9]*' gpurun_out/bench_ab.log)"
done
