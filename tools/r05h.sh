# encoder: GEMM / encoder parity on the new build, then Mode A A/B vs the previous encoder
set -o pipefail
mkdir -p gpurun_out/r05h
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_encoder.py tests/test_gpu_mode_a_f64.py > gpurun_out/r05h/tests.log 2>&1
rt=$?; echo "tests rc=$rt"; tail -4 gpurun_out/r05h/tests.log
[ $rt -eq 0 ] || exit $rt
for rep in 1 2; do
  for lib in two-tower-model-v2_amd/lib/libtwotower_hip.so two-tower-model-v2_amd/lib/variants/lib_encold.so; do
    TWOTOWER_HIP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --steps 3 --mode-a-steps 4 > gpurun_out/r05h/b.json 2>/dev/null || exit 1
    python -c "
import json,sys; d=json.loads(open('gpurun_out/r05h/b.json').read().strip().splitlines()[-1]); m=d['mode_a']
print(sys.argv[1].split('/')[-1], 'mode_a %.1f buyers/s  %.2f ms/step (1 stream %.1f, 2 streams %.1f)' % (m['value'], m['ms_per_step'], m['buyers_per_s_one_stream'], m['buyers_per_s_two_streams']))" $lib
  done
done
