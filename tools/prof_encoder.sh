#!/bin/bash
# On the GPU box: rocprofv3 kernel trace of the item-tower encoder at the Mode A shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/encprof -o run --output-format csv -- python tools/bench_encoder.py --batch ${BATCH:-5120} --batches ${BATCHES:-3} > gpurun_out/encprof.log 2>&1 || exit $?
python tools/kernel_table.py gpurun_out/encprof/run_kernel_trace.csv
