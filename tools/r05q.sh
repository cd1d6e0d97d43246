# bigger per-query candidate buffers in both single passes: tests, A/B, counts
set -o pipefail
mkdir -p gpurun_out/r05q
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_i8.py tests/test_gpu_parity.py > gpurun_out/r05q/tests.log 2>&1
rt=$?; echo "tests rc=$rt"; tail -3 gpurun_out/r05q/tests.log
[ $rt -eq 0 ] || exit $rt
for rep in 1 2; do
for lib in lib/libtwotower_hip.so lib/variants/lib_bb0.so lib/variants/lib_prev.so; do
  TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/$lib timeout -k 10 180 python -u tools/bench_i8.py > gpurun_out/r05q/b.json 2>gpurun_out/r05q/b.err || exit 1
  python -c "
import json,sys; d=json.load(open('gpurun_out/r05q/b.json'))
print(sys.argv[1], ' '.join('nq%s bf16 %.4f (%.4f) i8 %.4f (stream %.4f) fb %d' % (q[2:], v['bf16']['ms_per_search'], v['bf16']['stream_ms'], v['i8']['ms_per_search'], v['i8']['stream_ms'], v['i8']['fallbacks_last']) for q, v in d.items() if q.startswith('nq')))" $lib
done
done
for v in clk clkbb0; do
for nq in 1 4; do
NQ=$nq TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/variants/lib_$v.so timeout -k 10 120 python -u tools/i8clk.py > gpurun_out/r05q/${v}_nq$nq.json 2>gpurun_out/r05q/clk.err || exit 1
python -c "import json; print('$v', json.dumps(json.load(open('gpurun_out/r05q/${v}_nq$nq.json'))))"
done
done
