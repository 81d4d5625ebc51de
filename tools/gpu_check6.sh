#!/bin/bash
# Round-6 check of the current tree: the GPU suite (verbose, so the log grows as tests finish),
# smoke, the default bench line with the batched MLP image pass off / on (interleaved, same box),
# and the fp16 bench line.  Usage: tools/gpu_check6.sh OUTDIR
out=$GRAFT_REPO_ROOT/gpurun_out/$1
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
for i in 1 2; do
  for v in 0 1; do
    timeout -k 10 300 env VAETEB_MLP_PREP_BATCH=$v python bench.py --no-cpu-baseline > $out/bench_prep${v}_$i.json 2> $out/bench_prep${v}_$i.err || exit $?
  done
done
timeout -k 10 300 python bench.py --no-cpu-baseline --precision fp16 > $out/bench_fp16.json 2> $out/bench_fp16.err
