#!/bin/bash
# head GEMM kernels: MFMA GPU tests, then the same-box library A/B with kernel stats of one B bench
TAG=$1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_model.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || exit 1
bash tools/gpu_libab.sh $TAG || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof.log 2>&1
