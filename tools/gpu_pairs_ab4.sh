#!/bin/bash
out=$GRAFT_REPO_ROOT/gpurun_out/pab4
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontend.py -q --tb=short -p no:cacheprovider --timeout 200 --timeout-method thread > $out/t_fe.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/pairs_micro.py 1,0,1,0 > $out/micro.txt 2>&1 || exit $?
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/b_h1_$i.json 2> $out/b_h1_$i.err || exit $?
done
