# int8 sample level (LDS-staged scales): large-batch + int8 + vector-db tests, then bench
set -o pipefail
mkdir -p gpurun_out/r05af
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_large_batch.py tests/test_gpu_i8.py tests/test_gpu_vectordb_reference.py > gpurun_out/r05af/tests.log 2>&1
rt=$?; echo "tests rc=$rt"; tail -3 gpurun_out/r05af/tests.log
[ $rt -eq 0 ] || exit $rt
timeout -k 10 600 python bench.py > gpurun_out/r05af/bench.log 2>&1 || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/r05af/bench.log').read().strip().splitlines()[-1]); s=d['summary']
print(json.dumps({k:s[k] for k in ('value','ms_per_step','filter_frac','filter_ms','search_minus_filter_ms','fallbacks','self_check_bad','mode_a_buyers_per_s','one_buyer_ms','api_calls_per_s_1_vs_4_threads','configs1_texts_per_s','configs1_api_chunks_texts_per_s')}))"
