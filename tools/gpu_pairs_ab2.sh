#!/bin/bash
# pair-kernel forms (0 full image; 1 half image, one-lane pass 3; 3 half image, four-lane pass 3):
# front-end + J6 tests, the micro benchmark, then the bench interleaved
out=$GRAFT_REPO_ROOT/gpurun_out/pab2
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_frontend.py tests/test_gpu_parity_s256.py::test_j6_config2_step_end_to_end_vs_oracle -s -v --tb=short -p no:cacheprovider --timeout 250 --timeout-method thread > $out/t.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/pairs_micro.py 0,1,3,1,0,3 > $out/micro.txt 2>&1 || exit $?
for i in 1 2; do
for h in 1 0 3; do
VAETEB_PAIRS_HALF=$h timeout -k 10 300 python bench.py --no-cpu-baseline > $out/b_h${h}_$i.json 2> $out/b_h${h}_$i.err || exit $?
done
done
