#!/bin/bash
# On the GPU box: one-buyer / small-batch search latency for each variant library
# (tools/exp_filter.sh builds them), twice each in alternating order; SMALLT phase lines too.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for so in two-tower-model-v2_amd/lib/variants/lib_*.so; do
    name=$(basename $so .so)
    TWOTOWER_HIP_LIB=$PWD/$so timeout -k 10 200 python tools/bench_latency.py --nq ${NQ:-1,8,32,256} --methods bf16 > gpurun_out/lat_$name.log 2>&1
    rc=$?
    echo "$name rep$rep rc=$rc $(tail -1 gpurun_out/lat_$name.log)"
    grep SMALLT gpurun_out/lat_$name.log | tail -1
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
