# in-process A/B of the re-rank / threshold variants, then the full GPU suite
set -o pipefail
mkdir -p gpurun_out/r05e
V=two-tower-model-v2_amd/lib/variants
timeout -k 10 300 python -u tools/ab_inproc.py --reps 16 --libs $V/lib_r4.so,$V/lib_r4r.so,$V/lib_tp.so,$V/lib_tpr.so > gpurun_out/r05e/ab.json 2> gpurun_out/r05e/ab.err
echo "ab rc=$?"; cat gpurun_out/r05e/ab.json; tail -3 gpurun_out/r05e/ab.err
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r05e/tests.log 2>&1
echo "tests rc=$?"; tail -15 gpurun_out/r05e/tests.log
