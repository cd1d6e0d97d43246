# int8 single pass up to 8 queries: tests (int8, filter parity, vector db), latency by nq, API threads
set -o pipefail
mkdir -p gpurun_out/r05v
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_i8.py tests/test_gpu_parity.py tests/test_gpu_vectordb_reference.py > gpurun_out/r05v/tests.log 2>&1
rt=$?; echo "tests rc=$rt"; tail -2 gpurun_out/r05v/tests.log
[ $rt -eq 0 ] || exit $rt
NQS=1,2,4,5,8,16 timeout -k 10 200 python -u tools/bench_i8.py > gpurun_out/r05v/b.json 2>gpurun_out/r05v/b.err || exit 1
python tools/show_i8.py gpurun_out/r05v/b.json main
timeout -k 10 300 python -u tools/bench_api.py > gpurun_out/r05v/api.json 2>gpurun_out/r05v/api.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r05v/api.json')); print(json.dumps(d['variants']))"
