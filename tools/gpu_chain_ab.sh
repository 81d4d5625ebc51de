#!/bin/bash
# Chained 4-layer LSTM launches (round 6): the LSTM tests, bit-identity of two bf16 training
# steps with and without the chaining (tools/lib_bitwise.py at the bench geometry), then the
# default bench with each setting, interleaved.  Usage: tools/gpu_chain_ab.sh OUTDIR
out=$GRAFT_REPO_ROOT/gpurun_out/$1
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_lstm16.py > $out/pytest_lstm.log 2>&1 || exit $?
for s in 64 256; do
  timeout -k 10 180 env LB_S=$s LB_B=256 python tools/lib_bitwise.py run $out/chain_s$s.json > $out/lb.log 2>&1 || exit $?
  timeout -k 10 180 env LB_S=$s LB_B=256 VAETEB_L16_CHAIN_FWD=0 VAETEB_L16_CHAIN_BWD=0 python tools/lib_bitwise.py run $out/pairs_s$s.json >> $out/lb.log 2>&1 || exit $?
  python tools/lib_bitwise.py compare $out/chain_s$s.json $out/pairs_s$s.json >> $out/bitwise.txt 2>&1
done
for i in 1 2; do
  for cfg in "0 0" "1 1" "0 1" "1 0"; do
    set -- $cfg
    timeout -k 10 300 env VAETEB_L16_CHAIN_FWD=$1 VAETEB_L16_CHAIN_BWD=$2 python bench.py --no-cpu-baseline > $out/bench_f$1b$2_$i.json 2> $out/bench_f$1b$2_$i.err || exit $?
  done
done
