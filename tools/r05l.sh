# int8 stream: which part of the compute costs (timing-only variants) + /retrieve threads A/B
set -o pipefail
mkdir -p gpurun_out/r05l
for lib in lib/libtwotower_hip.so lib/variants/lib_noapp.so lib/variants/lib_nolds.so lib/variants/lib_nomfma.so lib/variants/lib_nocomp.so; do
  TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/$lib timeout -k 10 180 python -u tools/bench_i8.py > gpurun_out/r05l/b.json 2>gpurun_out/r05l/b.err || exit 1
  python -c "
import json,sys; d=json.load(open('gpurun_out/r05l/b.json'))
print(sys.argv[1], ' '.join('nq%s i8 stream %.4f' % (q[2:], v['i8']['stream_ms']) for q, v in d.items() if q.startswith('nq')))" $lib
done
timeout -k 10 300 python -u tools/bench_api.py > gpurun_out/r05l/api.json 2>gpurun_out/r05l/api.err || exit 1
cat gpurun_out/r05l/api.json
