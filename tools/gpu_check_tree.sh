#!/bin/bash
# A tree check: the GPU suite, two bench lines (compare their ELBO with an earlier tree's for
# bit-identity), a kernel trace of the bench.  Usage: tools/gpu_check_tree.sh OUTDIR
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-check}
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
( while sleep 45; do date >> $out/heartbeat; done ) & hb=$!
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
kill $hb
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/b_$i.json 2> $out/b_$i.err || exit $?
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/prof.log 2>&1
