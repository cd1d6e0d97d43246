#!/bin/bash
# On the GPU box: 12-step kernel trace + HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE in
# separate runs, as MI355X_MICROARCH.md's rocprofv3 section prescribes) of the batched bench step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-extra --mode-a-buyers 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p12 -o run --output-format csv -- $B --steps 12 --warmup 2 > gpurun_out/p12.log 2>&1 || exit 3
tail -1 gpurun_out/p12.log | cut -c1-300
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- $B --steps 2 --warmup 1 > gpurun_out/pmc_fetch.log 2>&1 || exit 4
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- $B --steps 2 --warmup 1 > gpurun_out/pmc_write.log 2>&1 || exit 5
echo pmc done
