#!/bin/bash
# On the GPU box: encoder kernel table (rocprofv3 kernel trace, Mode A shape) + FETCH/WRITE PMC.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/prof_encoder.sh > gpurun_out/enc_table.txt 2>&1 || { tail -5 gpurun_out/enc_table.txt; exit 1; }
cat gpurun_out/enc_table.txt
CMD="python tools/bench_encoder.py --batch ${BATCH:-5120} --batches 1"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/encpmc_$c -o run --output-format csv -- $CMD > gpurun_out/encpmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/encpmc_$c.log; exit 1; }
done
python tools/pmc_table.py gpurun_out/encpmc_*/run_counter_collection.csv
