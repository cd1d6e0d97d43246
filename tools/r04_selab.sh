#!/bin/bash
# GPU box: select-path variants (lib/variants/lib_<v>.so): parity tests on the first, then
# bench_large_k alternated x2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/two-tower-model-v2_amd/lib/variants
set -- ${VS:-a b}
TWOTOWER_HIP_LIB=$V/lib_$1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu \
  -p no:cacheprovider --timeout 200 --timeout-method thread -k "select" > gpurun_out/selab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/selab_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in ${VS:-a b}; do
    TWOTOWER_HIP_LIB=$V/lib_$v.so timeout -k 10 200 python tools/bench_large_k.py --paths select \
      --nqs ${NQS:-1,32} --ks 1000 > gpurun_out/selab_${v}_$rep.json 2>&1 || exit 1
    echo "$v $(tail -1 gpurun_out/selab_${v}_$rep.json)"
  done
done
