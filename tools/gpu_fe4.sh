#!/bin/bash
# front-end kernels: parity tests, micro-benchmark, pair-kernel phase timeline
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_frontend.py > gpurun_out/fe4_test.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/fe_micro.py > gpurun_out/fe4_micro.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/pairs_phases.py 256 > gpurun_out/fe4_phases.log 2>&1 || exit $?
