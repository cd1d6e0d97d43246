# k_sample_i8: 64- vs 128-row chunks (tests on the default, in-process A/B)
set -o pipefail
mkdir -p gpurun_out/r05ag
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_large_batch.py tests/test_gpu_i8.py > gpurun_out/r05ag/tests.log 2>&1
rt=$?; echo "tests rc=$rt"; tail -2 gpurun_out/r05ag/tests.log
[ $rt -eq 0 ] || exit $rt
timeout -k 10 500 python -u tools/ab_inproc.py --i8 --libs two-tower-model-v2_amd/lib/libtwotower_hip.so,two-tower-model-v2_amd/lib/variants/lib_ch128.so --reps 12 > gpurun_out/r05ag/ab.json 2>gpurun_out/r05ag/ab.err || exit 1
cat gpurun_out/r05ag/ab.json
