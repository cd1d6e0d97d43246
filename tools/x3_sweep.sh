#!/bin/bash
# On the GPU box: x3 encoder throughput vs the persistent-GEMM threshold (TT_X3_BIG_MIN).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/two-tower-model-v2_amd/lib/variants/lib_tb.so
for v in ${VALS:-3 0}; do
  r=$(TWOTOWER_HIP_LIB=$L TT_X3_BIG_MIN=$v timeout -k 10 100 python tools/bench_encoder.py --prec x3 --batches 20 2>&1 | grep '^{') || exit 1
  echo "min=$v $r"
done
