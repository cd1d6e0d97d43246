set -u
mkdir -p gpurun_out
REPS=2 BENCH_ARGS="--steps 5 --warmup 2 --dim 768 --catalog 2000000" timeout -k 10 600 bash tools/bench_ab.sh > gpurun_out/ab.log 2>&1 || exit 3
cat gpurun_out/ab.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/tr1 -o run --output-format csv -- python tools/bench_small_search.py --reps 21 > gpurun_out/small.log 2>&1 || exit 4
tail -2 gpurun_out/small.log
