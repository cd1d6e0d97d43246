#!/bin/bash
# On the GPU box: SQ/TCC counter passes over one command (CMD), e.g.
#   CMD="python tools/bench_gemm.py --M 370761 --iters 2 --only 1152,384,0,0 --no-torch --no-ln"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-one}
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
            "SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM" \
            "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- $CMD > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
done
python tools/pmc_table.py gpurun_out/pmc_${TAG}_*/run_counter_collection.csv
