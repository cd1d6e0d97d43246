cd $GRAFT_REPO_ROOT
for so in two-tower-model-v2_amd/lib/variants/lib_*.so; do
  echo "$so"; TWOTOWER_HIP_LIB=$PWD/$so timeout -k 10 120 python tools/bench_gemm.py --M 370761 --iters 10 ${GEMM_ARGS:-} || exit $?
done
