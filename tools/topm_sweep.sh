#!/bin/bash
# On the GPU box: small-batch search latency, single-pass (topm) vs multi-level path, per nq.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/two-tower-model-v2_amd/lib/variants/lib_tb.so
for n in ${NQS:-1 2 4 8 16}; do
  for m in 1 0; do
    r=$(TWOTOWER_HIP_LIB=$L TT_FILTER_TOPM=$m timeout -k 10 100 python tools/bench_small_search.py --nq $n 2>&1 | grep '^{') || exit 1
    echo "nq=$n topm=$m $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["prepared"]["events_ms"], d["b2b_ms"])')"
  done
done
