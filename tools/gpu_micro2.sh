#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_resmlp.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_mlp.log 2>&1
rc=$?; echo "mlp rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python tools/mlp_micro.py > gpurun_out/micro.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/microprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/mlp_micro.py > $GRAFT_REPO_ROOT/gpurun_out/microprof.log 2>&1
