#!/bin/bash
# round-6 evidence, part 2 (after the profiles are committed, so the bench lines read them): the GPU
# suite (verbose; a heartbeat while the host-side oracle ensembles run), smoke, the bench lines
# (default c2, c4, c5, DDP probe, literal J=6, fp16)
out=$GRAFT_REPO_ROOT/gpurun_out/r06final
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
( while sleep 45; do date >> $out/heartbeat; done ) & hb=$!
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
kill $hb
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench_default.err || exit $?
timeout -k 10 300 python bench.py --workload c4 > $out/bench_c4.json 2> $out/bench_c4.err || exit $?
timeout -k 10 300 python bench.py --workload c5 > $out/bench_c5.json 2> $out/bench_c5.err || exit $?
timeout -k 10 300 python bench.py --ddp-probe --no-cpu-baseline > $out/bench_ddp_probe.json 2> $out/bench_ddp_probe.err || exit $?
timeout -k 10 300 python bench.py --frontend j6 --no-cpu-baseline > $out/bench_j6.json 2> $out/bench_j6.err || exit $?
timeout -k 10 300 python bench.py --precision fp16 --no-cpu-baseline > $out/bench_fp16.json 2> $out/bench_fp16.err
