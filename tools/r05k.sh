# int8 stream without compute (timing-only variant) vs main; bench single-buyer leg with the int8 pass
set -o pipefail
mkdir -p gpurun_out/r05k
for lib in lib/libtwotower_hip.so lib/variants/lib_nocomp.so; do
  TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/$lib timeout -k 10 180 python -u tools/bench_i8.py > gpurun_out/r05k/b.json 2>gpurun_out/r05k/b.err || exit 1
  python -c "
import json,sys; d=json.load(open('gpurun_out/r05k/b.json'))
print(sys.argv[1], ' '.join('nq%s bf16 %.4f i8 %.4f (stream %.4f) fb %d' % (q[2:], v['bf16']['ms_per_search'], v['i8']['ms_per_search'], v['i8']['stream_ms'], v['i8']['fallbacks_last']) for q, v in d.items() if q.startswith('nq')))" $lib
done
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --mode-a-buyers 0 --no-extra > gpurun_out/r05k/bench.json 2>gpurun_out/r05k/bench.err || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/r05k/bench.json').read().strip().splitlines()[-1]); print(json.dumps(d['summary'])); sb=d['single_buyer_search']; print({k: v for k, v in sb.items() if 'int8' in k or 'bf16' in k or k=='ms_per_search'})"
