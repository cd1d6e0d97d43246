#!/bin/bash
# On the GPU box: batched-step A/B of bench.py over lib/variants/lib_*.so (alternating, xREPS).
#   REPS=3 BENCH_ARGS="--steps 20" bash tools/bench_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for so in two-tower-model-v2_amd/lib/variants/lib_*.so; do
    name=$(basename $so .so)
    TWOTOWER_HIP_LIB=$PWD/$so timeout -k 10 180 python bench.py --no-cpu-baseline --no-extra \
      ${BENCH_ARGS:---steps 20 --warmup 3} > gpurun_out/ab_${name}_$rep.json 2>&1 || exit 1
    python - "$name" gpurun_out/ab_${name}_$rep.json <<'EOF'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1], "ms/step %.3f" % d["ms_per_step"], "search %.3f" % r["search_ms"],
      "full %.3f" % r["kernel_ms"], "fallbacks", r["fallback_queries_last_step"],
      "self_check", d["self_check"]["mismatched_queries"], flush=True)
EOF
  done
done
