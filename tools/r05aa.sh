# int8 sample level of the batched search: large-batch parity (with / without), then A/B
set -o pipefail
mkdir -p gpurun_out/r05aa
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_large_batch.py > gpurun_out/r05aa/tests.log 2>&1
rt=$?; echo "tests rc=$rt"; tail -3 gpurun_out/r05aa/tests.log
[ $rt -eq 0 ] || exit $rt
timeout -k 10 300 python -u tools/ab_sample_i8.py > gpurun_out/r05aa/ab.json 2>gpurun_out/r05aa/ab.err || exit 1
cat gpurun_out/r05aa/ab.json
