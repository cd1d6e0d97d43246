# k_select_reg bound + compaction: filter parity tests, in-process A/B on configs[2]
set -o pipefail
mkdir -p gpurun_out/r05y
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_vectordb_reference.py > gpurun_out/r05y/tests.log 2>&1
rt=$?; echo "tests rc=$rt"; tail -2 gpurun_out/r05y/tests.log
[ $rt -eq 0 ] || exit $rt
timeout -k 10 400 python -u tools/ab_inproc.py --libs two-tower-model-v2_amd/lib/libtwotower_hip.so,two-tower-model-v2_amd/lib/variants/lib_sb0.so --reps 12 > gpurun_out/r05y/ab.json 2>gpurun_out/r05y/ab.err || exit 1
cat gpurun_out/r05y/ab.json
