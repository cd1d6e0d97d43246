#!/bin/bash
# GPU box, round 5 late build (small-batch query image): full -m gpu suite, smoke, bench.py, then the 12-step kernel trace of
# the batched step and its PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) -- each step time-limited,
# the session stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/r05q_$name.log" 2>&1
  local rc=$?
  tail -3 "gpurun_out/r05q_$name.log" | cut -c1-400
  echo "=== $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
if [ -z "${SKIP_TESTS:-}" ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
fi
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
[ -n "${BENCH_ONLY:-}" ] && exit 0
B="python bench.py --no-cpu-baseline --no-extra --mode-a-buyers 0"
step p12 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05q_p12 -o run --output-format csv -- $B --steps 12 --warmup 2
step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/r05q_pmc_fetch -o run --output-format csv -- $B --steps 2 --warmup 1
step pmc_write 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/r05q_pmc_write -o run --output-format csv -- $B --steps 2 --warmup 1
step pmc_sq 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/r05q_pmc_sq -o run --output-format csv -- $B --steps 2 --warmup 1
echo "prof done"
