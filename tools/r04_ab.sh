#!/bin/bash
# GPU box: encoder tests on lib_n (tools/ab_enc_build.sh), then x3 encode timings of lib_o vs
# lib_n alternated (B = 256 and 5120), then a kernel trace of lib_n at B = 256.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/two-tower-model-v2_amd/lib/variants
TWOTOWER_HIP_LIB=$V/lib_n.so timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder.py -x -q -m gpu \
  -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for B in 256 5120; do
    NB=$([ $B = 256 ] && echo 60 || echo 6)
    for v in o n; do
      TWOTOWER_HIP_LIB=$V/lib_$v.so timeout -k 10 180 python tools/bench_encoder.py --prec ${PREC:-x3} --batch $B \
        --batches $NB > gpurun_out/ab_${v}_${B}_$rep.json 2>&1 || exit 1
      echo "$v B=$B $(tail -1 gpurun_out/ab_${v}_${B}_$rep.json | cut -c1-150)"
    done
  done
done
TWOTOWER_HIP_LIB=$V/lib_n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab -o run \
  --output-format csv -- python tools/bench_encoder.py --prec x3 --batch ${PROF_B:-256} --batches ${PROF_NB:-20} > gpurun_out/prof_ab.log 2>&1 || exit 1
echo done
