#!/bin/bash
# On the GPU box: rocprofv3 kernel trace of tools/bench_small_search.py per lib variant
# (lib/variants/lib_*.so); per-kernel table -> gpurun_out/pv_<name>.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
for so in two-tower-model-v2_amd/lib/variants/lib_*.so; do
  name=$(basename $so .so)
  (cd /tmp && export TMPDIR=/tmp && TWOTOWER_HIP_LIB=$R/$so timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/pv_$name -o run -- python $R/tools/bench_small_search.py ${SMALL_ARGS:-} > $R/gpurun_out/pv_$name.log 2>&1) || exit 1
  python tools/db_kernels.py gpurun_out/pv_$name/run_results.db > gpurun_out/pv_$name.txt 2>&1
  echo "== $name"; head -4 gpurun_out/pv_$name.txt
  rm -rf gpurun_out/pv_$name
done
