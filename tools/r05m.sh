# cycle split of the int8 stream's tile loop (timing build)
set -o pipefail
mkdir -p gpurun_out/r05m
for nq in 1 4; do
NQ=$nq TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/variants/lib_clk.so timeout -k 10 120 python -u tools/i8clk.py > gpurun_out/r05m/clk_nq$nq.json 2>gpurun_out/r05m/clk.err || exit 1
cat gpurun_out/r05m/clk_nq$nq.json
done
