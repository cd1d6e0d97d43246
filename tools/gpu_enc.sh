set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_embedding_encoder.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/enc_tests.log 2>&1; rc=$?
tail -3 gpurun_out/enc_tests.log
[ $rc -ne 0 ] && exit $rc
for v in 1 0; do
  TT_GEMM_LN=$v timeout -k 10 120 python tools/bench_encoder.py --batch 5120 --batches 10 || exit $?
  TT_GEMM_LN=$v timeout -k 10 120 python tools/bench_encoder.py --batch 256 --batches 20 || exit $?
done
