#!/bin/bash
# GPU box: exact16 with its row loads issued before the MFMA chain -- k_final_small phases,
# small-batch latencies, then the GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/variants/lib_s9.so timeout -k 10 120 python tools/blktime_small.py --nq 32 > gpurun_out/r05p_blk_s9.json 2>&1 || exit 1
for nq in 16 32 256; do
  echo "$nq $(timeout -k 10 120 python tools/bench_small_search.py --nq $nq --modeb --reps 100 2>/dev/null | tail -1)" >> gpurun_out/r05p_small.txt || exit 1
done
NQS=1,8 timeout -k 10 200 python tools/bench_i8.py > gpurun_out/r05p_i8.json 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05p_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05p_tests.log; exit $rc
