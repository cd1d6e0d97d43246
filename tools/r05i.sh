# int8 single pass: parity tests, then latency vs bf16
set -o pipefail
mkdir -p gpurun_out/r05i
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_i8.py > gpurun_out/r05i/tests.log 2>&1
rt=$?; echo "tests rc=$rt"; grep -E "PASS|FAIL|Error|error" gpurun_out/r05i/tests.log | head -30; tail -30 gpurun_out/r05i/tests.log | grep -v "^$" | tail -25
[ $rt -eq 0 ] || exit $rt
timeout -k 10 200 python -u tools/bench_i8.py > gpurun_out/r05i/bench_i8.json 2> gpurun_out/r05i/bench_i8.err
echo "bench rc=$?"; cat gpurun_out/r05i/bench_i8.json; tail -3 gpurun_out/r05i/bench_i8.err
