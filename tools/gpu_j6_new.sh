#!/bin/bash
out=$GRAFT_REPO_ROOT/gpurun_out/j6new
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity_s256.py tests/test_gpu_frontend.py -s -v --tb=short -p no:cacheprovider --timeout 300 --timeout-method thread > $out/t.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
VAETEB_PAIRS_HALF=0 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity_s256.py::test_j6_config2_step_end_to_end_vs_oracle -s -q --tb=short -p no:cacheprovider --timeout 150 --timeout-method thread > $out/t_h0.log 2>&1
