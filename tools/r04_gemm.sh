#!/bin/bash
# GPU box: encoder GEMM tests, then the GEMM microbench A/B over timing-build variants
# (lib_t: TT_GEMM_PP=0 -> k_gemm_wide, =1 -> k_gemm_pp; lib_b2 / lib_np: k_gemm_pp with 2
# barriers per K-tile / without s_setprio), alternating x2, and the encode benchmark.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/two-tower-model-v2_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder.py -x -q -m gpu -p no:cacheprovider \
  --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/enc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/enc_tests.log; [ $rc -eq 0 ] || exit $rc
# the pp kernel's correctness (timing build, pp on)
TWOTOWER_HIP_LIB=$V/lib_b2.so TT_GEMM_PP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder.py -x -q -m gpu -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "gemm or encoder" > gpurun_out/enc_tests_pp.log 2>&1
rc=$?; tail -3 gpurun_out/enc_tests_pp.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in "t 0" "t 1" "b2 1" "np 1"; do
    set -- $v
    TWOTOWER_HIP_LIB=$V/lib_$1.so TT_GEMM_PP=$2 timeout -k 10 180 python tools/bench_gemm_pp.py > gpurun_out/gpp_$1$2_$rep.json 2>&1 || exit 1
    echo "$v $(tail -1 gpurun_out/gpp_$1$2_$rep.json)"
  done
done
for B in 256 5120; do
  NB=$([ $B = 256 ] && echo 60 || echo 6)
  for v in "x3 t 0" "x3 t 1" "x3 b2 1" "bf16 t 0" "bf16 b2 1"; do
    set -- $v
    TWOTOWER_HIP_LIB=$V/lib_$2.so TT_GEMM_PP=$3 timeout -k 10 180 python tools/bench_encoder.py --prec $1 --batch $B --batches $NB \
      > gpurun_out/enc_$1_$2$3_$B.json 2>&1 || exit 1
    echo "$v B=$B $(tail -1 gpurun_out/enc_$1_$2$3_$B.json)"
  done
done
echo done
