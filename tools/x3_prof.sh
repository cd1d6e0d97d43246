#!/bin/bash
# On the GPU box: rocprof kernel table of the x3 encoder per TT_X3_BIG_MIN value.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
L=$R/two-tower-model-v2_amd/lib/variants/lib_tb.so
for v in ${VALS:-3 0}; do
  (cd /tmp && export TMPDIR=/tmp && TWOTOWER_HIP_LIB=$L TT_X3_BIG_MIN=$v timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/x3p_$v -o run -- python $R/tools/bench_encoder.py --prec x3 --batches 10 > /dev/null 2>&1) || exit 1
  echo "== min=$v"; python tools/db_kernels.py gpurun_out/x3p_$v/run_results.db | head -5
  python - "$v" <<'PY'
import sqlite3, collections, sys
c = sqlite3.connect(f"gpurun_out/x3p_{sys.argv[1]}/run_results.db")
d = collections.defaultdict(list)
for name, gx, s, e in c.execute("select name, grid_x, start, end from kernels"):
    if "k_gemm" in name:
        d[(name.split("(")[0][-45:], gx)].append((e - s) / 1e3)
for k, v in sorted(d.items()):
    print(k, len(v), round(sum(v) / len(v), 1))
PY
  rm -rf gpurun_out/x3p_$v
done
