# full GPU suite on the current build, then the block timeline and the re-rank A/B
set -o pipefail
mkdir -p gpurun_out/r05d
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05d/smoke.log 2>&1
echo "smoke rc=$?"; tail -2 gpurun_out/r05d/smoke.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r05d/tests.log 2>&1
rt=$?
echo "tests rc=$rt"; tail -15 gpurun_out/r05d/tests.log
[ $rt -eq 0 ] || [ $rt -eq 1 ] || exit $rt
bash tools/r05c.sh
REPS=2 BENCH_ARGS="--steps 20 --warmup 3 --mode-a-buyers 0" timeout -k 10 400 bash tools/bench_ab.sh
