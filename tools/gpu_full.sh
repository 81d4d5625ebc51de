#!/bin/bash
# full GPU test suite, then default bench + GPU-only probe + GPU-bound kernel trace
TAG=$1; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 && \
bash tools/gpu_step_probe.sh $TAG
