set -o pipefail
mkdir -p gpurun_out/r05c
TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/exp/lib_blk.so timeout -k 10 120 python -u tools/blktime.py > gpurun_out/r05c/blktime.json 2> gpurun_out/r05c/blktime.err
echo "blktime rc=$?"
cat gpurun_out/r05c/blktime.json
