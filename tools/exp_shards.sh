#!/bin/bash
# On the GPU box: per variant library, the W=8 staged-shard emulation + the 1-GPU bench leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for so in two-tower-model-v2_amd/lib/variants/lib_*.so; do
  name=$(basename $so .so)
  TWOTOWER_HIP_LIB=$PWD/$so timeout -k 10 200 python tools/emulate_shards.py --world ${WORLD:-8} > gpurun_out/emu_$name.log 2>&1 || exit 1
  TWOTOWER_HIP_LIB=$PWD/$so timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --mode-a-buyers 0 --steps 3 --warmup 1 > gpurun_out/exp_$name.log 2>&1 || exit 1
  echo "$name $(grep -o '"staged_per_rank_ms": [0-9.]*\|"full": [0-9.]*' gpurun_out/emu_$name.log | tr '\n' ' ') $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/exp_$name.log)"
done
