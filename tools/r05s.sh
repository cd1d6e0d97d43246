# single passes for larger batches (timing builds) and the pure int8 stream with 4 / 5 slots
set -o pipefail
mkdir -p gpurun_out/r05s
run() {  # lib nqs i8max
  NQS=$2 I8MAX=$3 TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/$1 timeout -k 10 180 python -u tools/bench_i8.py > gpurun_out/r05s/b.json 2>gpurun_out/r05s/b.err || return 1
  python tools/show_i8.py gpurun_out/r05s/b.json $1
}
for rep in 1 2; do
run lib/libtwotower_hip.so 1,4,8,16 4 || exit 1
run lib/variants/lib_q8.so 1,4,8 8 || exit 1
run lib/variants/lib_q16.so 1,4,8,16 16 || exit 1
run lib/variants/lib_nocomp.so 1 4 || exit 1
run lib/variants/lib_nocomp5.so 1 4 || exit 1
done
