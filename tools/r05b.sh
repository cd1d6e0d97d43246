set -o pipefail
mkdir -p gpurun_out/r05b
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05b/smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_encoder.py tests/test_gpu_mode_a_f64.py tests/test_gpu_embedding_encoder.py tests/test_gpu_vectordb_reference.py tests/test_gpu_parity.py -k "envelope or head_vs or end_to_end or mode_a or encode_items or retrieve or plant or corrupt or persistent_ring" > gpurun_out/r05b/tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05b/smoke.log
tail -25 gpurun_out/r05b/tests.log
exit $rc
