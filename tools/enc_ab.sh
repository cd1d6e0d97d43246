#!/bin/bash
# On the GPU box: encoder A/B between lib/variants/lib_<name>.so builds (VARS), alternating, at
# BATCH texts per batch (configs[1]: 256; Mode A: 5120).  Extra env per variant: name=ENV=VAL.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in ${VARS:-prev new}; do
    lib=${v%%=*}; envs=""
    [ "$lib" != "$v" ] && envs=${v#*=}
    env $envs TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/variants/lib_$lib.so timeout -k 10 120 \
      python tools/bench_encoder.py --batch ${BATCH:-256} --batches ${BATCHES:-60} > gpurun_out/encab_$rep.json 2>&1 || exit 1
    echo "$v $(tail -1 gpurun_out/encab_$rep.json)"
  done
done
