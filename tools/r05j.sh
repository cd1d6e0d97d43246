#!/bin/bash
# GPU box: small-batch sample level ring depth (TT_RING_PD_S0 3 / 4 / 5) -- block phases, the
# one-search latency at 16 / 32 / 256 queries, and the parity suite on the deepest variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$PWD/two-tower-model-v2_amd/lib/variants
for v in s0 s0p5; do
  TWOTOWER_HIP_LIB=$V/lib_$v.so timeout -k 10 120 python tools/blktime_small.py --nq 32 > gpurun_out/r05j_blk_$v.json 2>&1 || exit 1
done
for rep in 1 2; do
  for v in base p4 p5; do
    for nq in 16 32 256; do
      echo "$v $nq $(TWOTOWER_HIP_LIB=$V/lib_$v.so timeout -k 10 120 python tools/bench_small_search.py --nq $nq --modeb --reps 100 2>/dev/null | tail -1)" >> gpurun_out/r05j_ab.txt || exit 1
    done
  done
done
TWOTOWER_HIP_LIB=$V/lib_p5.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vectordb_reference.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r05j_p5_tests.log 2>&1
tail -2 gpurun_out/r05j_p5_tests.log
