# serving path: coalescing + cached arguments -- vector DB tests, then the one-buyer API numbers
set -o pipefail
mkdir -p gpurun_out/r05g
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_vectordb_reference.py > gpurun_out/r05g/tests.log 2>&1
rt=$?; echo "tests rc=$rt"; tail -6 gpurun_out/r05g/tests.log
[ $rt -eq 0 ] || exit $rt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra --mode-a-buyers 0 > gpurun_out/r05g/bench.json 2> gpurun_out/r05g/bench.err
echo "bench rc=$?"
python -c "
import json; d=json.loads(open('gpurun_out/r05g/bench.json').read().strip().splitlines()[-1]); sb=d['single_buyer_search']
print({k: v for k, v in sb.items() if 'api' in k and 'is' not in k}, d['summary']['one_buyer_ms'])"
