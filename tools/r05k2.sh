#!/bin/bash
# GPU box: is the small-batch sample level's 15 us before its first tile the strided rows'
# address translation?  Block phases with the strided sample (s0) vs the first n_sample rows
# read contiguously (s0c, timing only), the full level's phases (s2), and the search latency.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$PWD/two-tower-model-v2_amd/lib/variants
for v in s0 s0c s2; do
  TWOTOWER_HIP_LIB=$V/lib_$v.so timeout -k 10 120 python tools/blktime_small.py --nq 32 > gpurun_out/r05k2_blk_$v.json 2>&1 || exit 1
done
for rep in 1 2; do
  for v in base c; do
    for nq in 32 256; do
      echo "$v $nq $(TWOTOWER_HIP_LIB=$V/lib_$v.so timeout -k 10 120 python tools/bench_small_search.py --nq $nq --modeb --reps 100 2>/dev/null | tail -1)" >> gpurun_out/r05k2_ab.txt || exit 1
    done
  done
done
echo done
