#!/bin/bash
# Round-6 check of the current tree: the GPU suite (verbose, so the log grows as tests finish),
# smoke, the default bench line and the fp16 bench line.  Usage: tools/gpu_check6.sh OUTDIR
out=$GRAFT_REPO_ROOT/gpurun_out/$1
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench_default.json 2> $out/bench_default.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --precision fp16 > $out/bench_fp16.json 2> $out/bench_fp16.err
# BatchNorm backward micro A/B (same bits expected): column partials 4 / 8 loads in flight,
# BN-gradient rows in 64 / 256-row blocks
for cfg in "4 64" "8 256" "4 64" "8 256"; do
  set -- $cfg
  echo "== COLP_U $1 BNX16_ROWS $2" >> $out/bn_ab.log
  VAETEB_COLP_U=$1 VAETEB_BNX16_ROWS=$2 timeout -k 10 120 python tools/bn_micro.py >> $out/bn_ab.log 2>&1 || exit $?
done
