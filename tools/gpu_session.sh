#!/bin/bash
# Runs on the GPU box (via gpurun): parity tests, smoke, bench, rocprof kernel trace.
# Every GPU step has its own time limit; a crash/timeout (rc not 0/1) stops the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-tests smoke bench prof}"
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    tests) if [ -n "${PYTEST_K:-}" ]; then
             run pytest_gpu 900 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "$PYTEST_K"
           else
             run pytest_gpu 900 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
           fi ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ${BENCH_ARGS:-} ;;
    bench_f32) run bench_f32 600 python bench.py --method f32 --no-cpu-baseline ${BENCH_ARGS:-} ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --steps ${PROF_STEPS:-3} --warmup ${PROF_WARMUP:-1} ${BENCH_ARGS:-} ;;
    pmc)   run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 2 --warmup 1 ${BENCH_ARGS:-}
           run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 2 --warmup 1 ${BENCH_ARGS:-} ;;
    sq)    run pmc_sq1 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace -d gpurun_out/pmc_sq1 -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 ${BENCH_ARGS:-}
           run pmc_sq2 600 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_sq2 -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 ${BENCH_ARGS:-} ;;
    list)  run pmc_list 120 rocprofv3 -L ;;
  esac
done
echo "session done"
