#!/bin/bash
# On the GPU box: one-buyer latency A/B over lib/variants/lib_*.so (alternating, x2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for so in two-tower-model-v2_amd/lib/variants/lib_*.so; do
    name=$(basename $so .so)
    TWOTOWER_HIP_LIB=$PWD/$so timeout -k 10 120 python tools/bench_small_search.py ${SMALL_ARGS:-} > gpurun_out/small_$name.json 2>&1 || exit 1
    echo "$name $(tail -1 gpurun_out/small_$name.json)"
  done
done
