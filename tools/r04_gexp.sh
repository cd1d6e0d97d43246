#!/bin/bash
# GPU box: GEMM microbench over timing-build variants (lib/variants/lib_<v>.so), alternated x2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/two-tower-model-v2_amd/lib/variants
for rep in 1 2; do
  for v in ${VS:-t h e}; do
    TWOTOWER_HIP_LIB=$V/lib_$v.so timeout -k 10 180 python tools/bench_gemm_x3i.py --M ${MS:-370761,18340} --iters 20 \
      > gpurun_out/gexp_${v}_$rep.json 2>&1 || exit 1
    echo "$v $(tail -1 gpurun_out/gexp_${v}_$rep.json)"
  done
done
