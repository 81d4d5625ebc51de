#!/bin/bash
# the whole GPU suite (verbose, so the log grows as tests finish; a heartbeat file while the
# CPU-side oracle ensembles of the B = 256 tests run), smoke, the default bench line.
# Usage: tools/gpu_suite.sh OUTDIR
out=$GRAFT_REPO_ROOT/gpurun_out/$1
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
( while sleep 45; do date >> $out/heartbeat; done ) & hb=$!
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
kill $hb
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench_default.err
