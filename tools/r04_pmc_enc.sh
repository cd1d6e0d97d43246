#!/bin/bash
# GPU box: two SQ counter passes over the x3 encoder at Mode A size (bench_encoder, B = 5120).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace -d gpurun_out/pmce_$i -o run --output-format csv -- python tools/bench_encoder.py --prec x3 --batch ${B:-5120} --batches 2 > gpurun_out/pmce_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmce_$i.log; exit 1; }
done
python tools/pmc_table.py gpurun_out/pmce_*/run_counter_collection.csv > gpurun_out/pmce_table.txt
head -120 gpurun_out/pmce_table.txt
