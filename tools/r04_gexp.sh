#!/bin/bash
# GPU box: GEMM microbench over timing-build variants (lib/variants/lib_<v>.so), alternated x2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/two-tower-model-v2_amd/lib/variants
for rep in 1 2; do
  for v in ${VS:-t h e}; do
    if [ -z "${NOGEMM:-}" ]; then
      TWOTOWER_HIP_LIB=$V/lib_$v.so timeout -k 10 180 python tools/bench_gemm_x3i.py --M ${MS:-370761,18340} --iters 20 \
        > gpurun_out/gexp_${v}_$rep.json 2>&1 || exit 1
      echo "$v $(tail -1 gpurun_out/gexp_${v}_$rep.json)"
    fi
    if [ -n "${ENC:-}" ]; then
      for B in 256 5120; do
        NB=$([ $B = 256 ] && echo 60 || echo 6)
        TWOTOWER_HIP_LIB=$V/lib_$v.so timeout -k 10 180 python tools/bench_encoder.py --prec x3 --batch $B \
          --batches $NB > gpurun_out/genc_${v}_${B}_$rep.json 2>&1 || exit 1
        echo "$v enc B=$B $(tail -1 gpurun_out/genc_${v}_${B}_$rep.json | cut -c1-120)"
      done
    fi
  done
done
