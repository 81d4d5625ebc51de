#!/bin/bash
# full GPU test suite, then the same-box library A/B (tools/gpu_libab.sh)
TAG=$1; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || exit 1
bash tools/gpu_libab.sh $TAG "$@"
