#!/bin/bash
# GPU box: filter parity tests (product build), then bench A/B of the full level's query
# loading: lib_e0 + TT_FILTER_Q16=0 (round-3 order), lib_t + Q16=0 (ring DMA first), lib_t +
# Q16=1 (bf16 query image), alternating x2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/two-tower-model-v2_amd/lib/variants
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_batch.py tests/test_gpu_sharded_index.py tests/test_gpu_configs4.py -x -q -m gpu -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/flt_tests.log 2>&1
rc=$?; tail -3 gpurun_out/flt_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in "e0 0" "t 0" "t 1"; do
    set -- $v
    TWOTOWER_HIP_LIB=$V/lib_$1.so TT_FILTER_Q16=$2 timeout -k 10 300 python bench.py --no-extra --no-cpu-baseline --mode-a-buyers 0 --steps 10 --warmup 2 > gpurun_out/fab_$1$2_$rep.json 2>&1 || exit 1
    python - "$v" gpurun_out/fab_$1$2_$rep.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r=d["roofline"]
print(sys.argv[1], "value %.0f ms/step %.3f kernel %.3f frac %.4f search %.3f fb %d check %s" % (d["value"], d["ms_per_step"], r["kernel_ms"], r["frac"], r["search_ms"], r["fallback_queries_last_step"], d["self_check"]["mismatched_queries"]))
PY
  done
done
echo done
