#!/bin/bash
# pair kernel A/B: direct HBM columns (default) vs LDS-staged product; front-end parity tests
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontend.py tests/test_gpu_api.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_fe.log 2>&1 && \
VAETEB_PAIRS_DIRECT=0 timeout -k 10 120 python tools/fe_micro.py > gpurun_out/fe_micro_staged.log 2>&1 && \
VAETEB_PAIRS_DIRECT=1 timeout -k 10 120 python tools/fe_micro.py > gpurun_out/fe_micro_direct.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/feprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/fe_micro.py > $GRAFT_REPO_ROOT/gpurun_out/feprof.log 2>&1
