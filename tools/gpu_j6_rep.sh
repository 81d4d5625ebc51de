#!/bin/bash
# the J=6 end-to-end test repeated per pair-kernel form (is its failure the form or intermittent?)
out=$GRAFT_REPO_ROOT/gpurun_out/j6rep
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
for i in 1 2 3; do
for h in 1 0; do
VAETEB_PAIRS_HALF=$h timeout -k 10 200 python -u -m pytest tests/test_gpu_parity_s256.py::test_j6_config2_step_end_to_end_vs_oracle -s -q --tb=line -p no:cacheprovider --timeout 150 --timeout-method thread > $out/t_h${h}_$i.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
done
