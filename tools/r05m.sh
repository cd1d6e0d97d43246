#!/bin/bash
# GPU box, round 5 late build (small batches through k_query_eps; branch-free int8 query
# coding in k_filter_topm_i8): GPU suite, then the small-batch latencies.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05m_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05m_tests.log; [ $rc -eq 0 ] || exit $rc
NQS=1,4,8 timeout -k 10 200 python tools/bench_i8.py > gpurun_out/r05m_i8.json 2>&1 || exit 1
for nq in 16 32 256; do
  echo "$nq $(timeout -k 10 120 python tools/bench_small_search.py --nq $nq --modeb --reps 100 2>/dev/null | tail -1)" >> gpurun_out/r05m_small.txt || exit 1
done
echo done
