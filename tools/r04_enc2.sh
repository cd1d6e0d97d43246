#!/bin/bash
# GPU box: encoder tests + x3 / bf16 encode timings + a kernel trace of the x3c configs[1] batch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder.py -x -q -m gpu -p no:cacheprovider \
  --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/enc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/enc_tests.log; [ $rc -eq 0 ] || exit $rc
for B in 256 5120; do
  NB=$([ $B = 256 ] && echo 60 || echo 6)
  for p in x3 bf16; do
    timeout -k 10 180 python tools/bench_encoder.py --prec $p --batch $B --batches $NB \
      > gpurun_out/enc_${p}_$B.json 2>&1 || exit 1
    echo "$p B=$B $(tail -1 gpurun_out/enc_${p}_$B.json)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_enc2 -o run --output-format csv \
  -- python tools/bench_encoder.py --prec x3 --batch 256 --batches 20 > gpurun_out/prof_enc2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_enc3 -o run --output-format csv \
  -- python tools/bench_encoder.py --prec x3 --batch 5120 --batches 3 > gpurun_out/prof_enc3.log 2>&1 || exit 1
echo done
