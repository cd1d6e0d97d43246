#!/bin/bash
# One GPU session on the box: bash tools/session.sh STEP [STEP ...]  (run through gpurun).
# Every step runs under its own time limit; the first failing step ends the session (no
# retries).  Outputs go to gpurun_out/<tag>/ (tag = $TAG, default "s").
set -o pipefail
TAG=${TAG:-s}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"

step() {  # name seconds command...
  local name=$1 secs=$2
  shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then
    echo "== $name FAILED rc=$rc"
    exit $rc
  fi
}

for s in "$@"; do
  case $s in
    gpu_tests) step gpu_tests 900 $PYT -m gpu tests ;;
    i8_tests) step i8_tests 400 $PYT -m gpu tests/test_gpu_i8.py tests/test_gpu_vectordb_reference.py ;;
    # the int8 single pass built with a 5-slot ring (timing build, tools/exp_build2.sh), its
    # parity cases only: round 5's unexplained illegal-address fault (tools/r05r.sh)
    sl5) TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/variants/lib_sl5.so \
           step sl5 300 $PYT -m gpu tests/test_gpu_i8.py -k "bit_exact or falls_back" ;;
    # round 5's r05r loop (tools/r05r.sh: bench_i8 over the 5-slot and no-compute timing
    # builds), once per library: which build raised the illegal address
    r05r_repro) for v in sl5 nocomp nocomp5; do
        TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/variants/lib_$v.so \
          step bench_i8_$v 180 python3 -u tools/bench_i8.py; done ;;
    train_prof) step train_prof 300 rocprofv3 --kernel-trace --stats --output-format csv \
                  -d "$OUT/train_prof" -o train -- python3 tools/train_step_prof.py ;;
    # the training step under timing builds (VARS = names under lib/variants), product lib first
    train_ab) for rep in 1 2; do for v in base ${VARS:-b512 b256 b2048}; do
        L=$PWD/two-tower-model-v2_amd/lib/variants/lib_$v.so; [ $v = base ] && L=$PWD/two-tower-model-v2_amd/lib/libtwotower_hip.so
        TWOTOWER_HIP_LIB=$L step train_ab_${v}_$rep 200 python3 tools/train_step_prof.py --json "$OUT/ab_${v}_$rep.json"
        python3 -c "import json; d=json.load(open('$OUT/ab_${v}_$rep.json')); print('$v $rep', round(d['bf16']['graph_inplace_inputs_ms'],4), round(d['f32']['graph_inplace_inputs_ms'],4))"
      done; done ;;
    train_bench) step train_bench 300 python3 tools/train_step_prof.py --json "$OUT/train.json" ;;
    trainer_tests) step trainer_tests 600 $PYT -m gpu tests/test_gpu_trainer.py tests/test_gpu_train.py tests/test_gpu_loss.py ;;
    debug_graph) step debug_graph 200 python3 -u tools/debug_graph_step.py ;;
    trainer_tests_nograph) step trainer_tests_nograph 600 $PYT -m gpu tests/test_gpu_trainer.py tests/test_gpu_train.py tests/test_gpu_loss.py -k "not graph_step" ;;
    enc_batch) step enc_batch 400 $PYT -s -m gpu tests/test_gpu_encoder.py -k large_batch ;;
    enc_prof) step enc_prof_5120 300 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$OUT/enc5120" -o run -- python3 tools/bench_encoder.py --prec x3 --batch 5120 --batches 3 &&
              step enc_prof_256 300 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$OUT/enc256" -o run -- python3 tools/bench_encoder.py --prec x3 --batch 256 --batches 20 ;;
    # A/B of a timing-switch (AB_ENV=NAME, values 0 / 1) on the timing build lib_tb.so: the
    # encoder's x3 tests under the switch, then bench_encoder alternating x2 at 5120 and 256
    enc_ab) L=$PWD/two-tower-model-v2_amd/lib/variants/lib_tb.so
        env TWOTOWER_HIP_LIB=$L $AB_ENV=1 timeout -k 10 400 $PYT -m gpu tests/test_gpu_encoder.py \
          -k "x3 or attention or large_batch" > "$OUT/enc_ab_tests.log" 2>&1 || { tail -5 "$OUT/enc_ab_tests.log"; exit 1; }
        tail -1 "$OUT/enc_ab_tests.log"
        for rep in 1 2; do for v in 0 1; do for b in 5120 256; do
          nb=$([ $b = 5120 ] && echo 3 || echo 20)
          env TWOTOWER_HIP_LIB=$L $AB_ENV=$v timeout -k 10 200 python3 tools/bench_encoder.py --prec x3 \
            --batch $b --batches $nb > "$OUT/ab_${v}_${b}_$rep.json" 2>/dev/null || exit 1
          echo "$AB_ENV=$v b=$b rep=$rep $(tail -1 $OUT/ab_${v}_${b}_$rep.json | cut -c1-120)"
        done; done; done ;;
    probe) step probe 120 ./tools/bin/stream_probe ;;
    i8r_tests) step i8r_tests 500 $PYT -m gpu tests/test_gpu_i8.py tests/test_gpu_vectordb_reference.py ;;
    i8r_bench) step i8r_bench 300 python3 -u tools/bench_i8.py ;;
    # the tiled stream's timing builds (tools/exp_build2.sh; VARS = names under lib/variants)
    i8r_ab) for v in ${VARS:-noapp nomfma d2 d3 d5}; do
        TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/variants/lib_$v.so NQS=1 I8VS=tiled,ring \
          step i8r_ab_$v 120 python3 -u tools/bench_i8.py
        python3 -c "import json,sys; t=open('$OUT/i8r_ab_$v.log').read(); d=json.loads(t[t.index('{'):]); print('$v', {k: round(r['stream_ms'], 4) for k, r in d['nq1'].items()})"
      done ;;
    # fixed costs vs bytes: the int8 streams at 4 catalog sizes (a linear fit of stream_ms)
    i8r_sizes) for nn in 16384 131072 500000 1000000; do
        N=$nn NQS=1 I8VS=tiled,ring,tiled,ring step i8r_size_$nn 120 python3 -u tools/bench_i8.py
        python3 -c "import json,sys; t=open('$OUT/i8r_size_$nn.log').read(); d=json.loads(t[t.index('{'):]); print('$nn', {k: round(r['stream_ms'], 4) for k, r in d['nq1'].items()})"
      done ;;
    i8r_clk) for nn in 1000000 16384; do
        N=$nn TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/variants/lib_clk.so \
          step i8r_clk_$nn 120 python3 -u tools/i8r_clk.py; cat "$OUT/i8r_clk_$nn.log"
      done ;;
    i8r_clk_nq) for nq in 1 16 32; do
        NQ=$nq TWOTOWER_HIP_LIB=$PWD/two-tower-model-v2_amd/lib/variants/lib_clk.so \
          step i8r_clk_nq$nq 120 python3 -u tools/i8r_clk.py
      done ;;
    i8r_prof) step i8r_prof 300 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$OUT/i8r_prof" -o run -- python3 tools/bench_i8.py ;;
    bench) step bench 600 python3 bench.py --steps 20 --warmup 5 ;;
    smoke) step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== session done"
