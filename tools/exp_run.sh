#!/bin/bash
# On the GPU box: time each variant's final-level filter kernel (bench.py kernel_ms).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for so in two-tower-model-v2_amd/lib/variants/lib_*.so; do
  name=$(basename $so .so)
  TWOTOWER_HIP_LIB=$PWD/$so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/exp_$name.log 2>&1
  rc=$?
  echo "$name rc=$rc $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/exp_$name.log) $(grep -o '"search_ms": [0-9.]*' gpurun_out/exp_$name.log) $(grep -o '"fallback_queries_last_step": [0-9]*' gpurun_out/exp_$name.log) $(grep -o '"value": [0-9.]*' gpurun_out/exp_$name.log | head -1) $(grep -o '"ms_per_search": [0-9.]*\|"full_level_ms": [0-9.]*' gpurun_out/exp_$name.log | tr '\n' ' ')"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
