#!/bin/bash
# GPU box: PMC passes over the x3i / bf16 GEMM microbenchmark at Mode A M (separate passes,
# one counter group each, under their own time limits).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for M in ${MS:-370761 18340}; do
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_SALU" \
            "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace -d gpurun_out/pmcg_${M}_$i -o run --output-format csv -- python tools/bench_gemm_x3i.py --M $M --iters 2 > gpurun_out/pmcg_${M}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmcg_${M}_$i.log; exit 1; }
done
python tools/pmc_table.py gpurun_out/pmcg_${M}_*/run_counter_collection.csv > gpurun_out/pmcg_table_$M.txt
done
head -60 gpurun_out/pmcg_table_*.txt
