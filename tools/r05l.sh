#!/bin/bash
# GPU box: small batches through k_query_eps (bf16 query image, TT_Q16_SMALL=1) vs the state
# folded into the first ring level (0) -- block phases of both ring levels, and the search
# latency at 16 / 32 / 64 / 256 queries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$PWD/two-tower-model-v2_amd/lib/variants
for v in s0 s2; do
  TWOTOWER_HIP_LIB=$V/lib_$v.so timeout -k 10 120 python tools/blktime_small.py --nq 32 > gpurun_out/r05l_blk_$v.json 2>&1 || exit 1
done
for rep in 1 2; do
  for v in off on; do
    for nq in 16 32 64 256; do
      echo "$v $nq $(TWOTOWER_HIP_LIB=$V/lib_$v.so timeout -k 10 120 python tools/bench_small_search.py --nq $nq --modeb --reps 100 2>/dev/null | tail -1)" >> gpurun_out/r05l_ab.txt || exit 1
    done
  done
done
echo done
