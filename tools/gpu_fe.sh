#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontend.py tests/test_gpu_api.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_fe.log 2>&1
rc=$?; echo "fe rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python tools/fe_micro.py > gpurun_out/fe_micro.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/feprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/fe_micro.py > $GRAFT_REPO_ROOT/gpurun_out/feprof.log 2>&1
