#!/bin/bash
# On the GPU box: SQ counters of the filter kernel for each variant in lib/variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for so in two-tower-model-v2_amd/lib/variants/lib_*.so; do
  name=$(basename $so .so)
  for set in "a:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" "b:SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "c:SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM"; do
    tag=${set%%:*}; ctrs=${set#*:}
    TWOTOWER_HIP_LIB=$PWD/$so timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace -d gpurun_out/sq_${name}_$tag -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 --mode-a-buyers 0 > gpurun_out/sq_${name}_$tag.log 2>&1
    rc=$?
    echo "$name $tag rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
