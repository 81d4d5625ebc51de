#!/bin/bash
# pair-kernel form 4 (one-thread pass 2) vs form 1, and the parity tests at form 1 (default)
out=$GRAFT_REPO_ROOT/gpurun_out/pab3
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity_s256.py -s -v --tb=short -p no:cacheprovider --timeout 300 --timeout-method thread > $out/t_parity.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
VAETEB_PAIRS_HALF=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_frontend.py -q --tb=short -p no:cacheprovider --timeout 200 --timeout-method thread > $out/t_fe4.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/pairs_micro.py 1,4,1,4 > $out/micro.txt 2>&1 || exit $?
for i in 1 2; do
for h in 1 4; do
VAETEB_PAIRS_HALF=$h timeout -k 10 300 python bench.py --no-cpu-baseline > $out/b_h${h}_$i.json 2> $out/b_h${h}_$i.err || exit $?
done
done
