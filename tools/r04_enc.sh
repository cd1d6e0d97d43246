#!/bin/bash
# GPU box: encoder x3c parity tests + x3c / x3 (split-in-loop) / bf16 encode timings at the
# configs[1] (256 texts) and Mode A (5120 texts) batch shapes, plus a rocprof kernel table of
# the x3c configs[1] batch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder.py -x -q -m gpu -p no:cacheprovider \
  --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/enc_tests.log 2>&1
rc=$?; tail -5 gpurun_out/enc_tests.log; [ $rc -eq 0 ] || exit $rc
for B in 256 5120; do
  NB=$([ $B = 256 ] && echo 60 || echo 6)
  for v in "x3 TT_X3C=1" "x3 TT_X3C=0" "bf16 TT_X3C=1"; do
    set -- $v
    env $2 timeout -k 10 180 python tools/bench_encoder.py --prec $1 --batch $B --batches $NB \
      > gpurun_out/enc_$1_$2_$B.json 2>&1 || exit 1
    echo "$v B=$B $(tail -1 gpurun_out/enc_$1_$2_$B.json)"
  done
done
if [ -n "${PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_enc -o run --output-format csv \
    -- python tools/bench_encoder.py --prec x3 --batch 256 --batches 20 > gpurun_out/prof_enc.log 2>&1 || exit 1
fi
echo done
