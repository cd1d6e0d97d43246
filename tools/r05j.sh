# int8 single pass: tests on the new swizzle, latency A/B (main vs old swizzle vs 5 slots), x2
set -o pipefail
mkdir -p gpurun_out/r05j
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_i8.py > gpurun_out/r05j/tests.log 2>&1
rt=$?; echo "tests rc=$rt"; tail -2 gpurun_out/r05j/tests.log
[ $rt -eq 0 ] || exit $rt
for rep in 1 2; do
for lib in lib/libtwotower_hip.so lib/variants/lib_swz0.so lib/variants/lib_sl5.so; do
  TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/$lib timeout -k 10 120 python -u tools/bench_i8.py > gpurun_out/r05j/b.json 2>/dev/null || exit 1
  python -c "
import json,sys; d=json.load(open('gpurun_out/r05j/b.json'))
print(sys.argv[1], ' '.join('nq%s bf16 %.4f i8 %.4f (stream %.4f) fb %d' % (q[2:], v['bf16']['ms_per_search'], v['i8']['ms_per_search'], v['i8']['stream_ms'], v['i8']['fallbacks_last']) for q, v in d.items() if q.startswith('nq')))" $lib
done
done
