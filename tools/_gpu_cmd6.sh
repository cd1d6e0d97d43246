set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_batch.py tests/test_gpu_configs4.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_lb.log 2>&1 || { tail -30 gpurun_out/pytest_lb.log; exit 3; }
tail -3 gpurun_out/pytest_lb.log
REPS=2 BENCH_ARGS="--steps 5 --warmup 2 --dim 768 --catalog 2000000" timeout -k 10 600 bash tools/bench_ab.sh > gpurun_out/ab.log 2>&1 || exit 4
cat gpurun_out/ab.log
