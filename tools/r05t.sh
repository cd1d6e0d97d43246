# shared tau bound across a block's compute waves: tests, A/B vs previous, cycle split
set -o pipefail
mkdir -p gpurun_out/r05t
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_i8.py tests/test_gpu_parity.py > gpurun_out/r05t/tests.log 2>&1
rt=$?; echo "tests rc=$rt"; tail -2 gpurun_out/r05t/tests.log
[ $rt -eq 0 ] || exit $rt
run() {
  NQS=$2 TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/$1 timeout -k 10 180 python -u tools/bench_i8.py > gpurun_out/r05t/b.json 2>gpurun_out/r05t/b.err || return 1
  python tools/show_i8.py gpurun_out/r05t/b.json $1
}
for rep in 1 2; do
run lib/libtwotower_hip.so 1,2,4 || exit 1
run lib/variants/lib_prev.so 1,2,4 || exit 1
done
for nq in 1 4; do
NQ=$nq TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/variants/lib_clk.so timeout -k 10 120 python -u tools/i8clk.py > gpurun_out/r05t/clk_nq$nq.json 2>gpurun_out/r05t/clk.err || exit 1
python -c "import json; print(json.dumps(json.load(open('gpurun_out/r05t/clk_nq$nq.json'))))"
done
