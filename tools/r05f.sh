# balanced partial-tile plan: in-process A/B (1M x 384, 2M x 768), block timeline, filter parity
set -o pipefail
mkdir -p gpurun_out/r05f
V=two-tower-model-v2_amd/lib/variants
timeout -k 10 300 python -u tools/ab_inproc.py --reps 16 --libs $V/lib_unb.so,$V/lib_bal.so > gpurun_out/r05f/ab384.json 2> gpurun_out/r05f/ab384.err
echo "ab384 rc=$?"; cat gpurun_out/r05f/ab384.json
timeout -k 10 300 python -u tools/ab_inproc.py --reps 8 --n 2000000 --dim 768 --libs $V/lib_unb.so,$V/lib_bal.so > gpurun_out/r05f/ab768.json 2> gpurun_out/r05f/ab768.err
echo "ab768 rc=$?"; cat gpurun_out/r05f/ab768.json
TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/exp/lib_blk.so timeout -k 10 120 python -u tools/blktime.py > gpurun_out/r05f/blktime.json 2> gpurun_out/r05f/blktime.err
echo "blktime rc=$?"; cat gpurun_out/r05f/blktime.json
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_large_batch.py tests/test_gpu_parity.py tests/test_gpu_configs4.py tests/test_gpu_sharded_index.py > gpurun_out/r05f/tests.log 2>&1
echo "tests rc=$?"; tail -5 gpurun_out/r05f/tests.log
