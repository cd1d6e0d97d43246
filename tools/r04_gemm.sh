#!/bin/bash
# GPU box: encoder GEMM tests, then the GEMM microbench A/B (TT_GEMM_PP=0/1, alternating x2)
# and the encode benchmark A/B at configs[1] / Mode A shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder.py -x -q -m gpu -p no:cacheprovider \
  --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/enc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/enc_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 0 1; do
    TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/variants/lib_t.so TT_GEMM_PP=$v timeout -k 10 180 python tools/bench_gemm_pp.py > gpurun_out/gpp_${v}_$rep.json 2>&1 || exit 1
    echo "pp=$v $(tail -1 gpurun_out/gpp_${v}_$rep.json)"
  done
done
for B in 256 5120; do
  NB=$([ $B = 256 ] && echo 60 || echo 6)
  for v in "x3 0" "x3 1" "bf16 0" "bf16 1"; do
    set -- $v
    TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/variants/lib_t.so TT_GEMM_PP=$2 timeout -k 10 180 python tools/bench_encoder.py --prec $1 --batch $B --batches $NB \
      > gpurun_out/enc_$1_pp$2_$B.json 2>&1 || exit 1
    echo "$v B=$B $(tail -1 gpurun_out/enc_$1_pp$2_$B.json)"
  done
done
echo done
