#!/bin/bash
# On the GPU box: encoder GEMM tests + microbenchmarks at the Mode A token count, for each
# TT_GEMM_BIG variant listed in VARIANTS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-1 2}; do
  TT_GEMM_BIG=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/gemm_tests_$v.log 2>&1 || { tail -30 gpurun_out/gemm_tests_$v.log; exit 1; }
  echo "variant $v: $(tail -1 gpurun_out/gemm_tests_$v.log)"
  TT_GEMM_BIG=$v timeout -k 10 120 python tools/bench_gemm.py --M 370761 --iters 10 || exit $?
  TT_GEMM_BIG=$v timeout -k 10 120 python tools/bench_encoder.py --batch 5120 --batches 10 || exit $?
done
