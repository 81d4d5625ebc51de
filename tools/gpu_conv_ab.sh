#!/bin/bash
# conv kernels: GPU conv tests, isolated decoder-conv trace, same-box bench A/B
TAG=$1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv_bf16.py tests/test_gpu_model.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || exit 1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/conv_micro.py > $GRAFT_REPO_ROOT/gpurun_out/$TAG/micro.txt 2>&1 ) || exit 1
bash tools/gpu_libab.sh $TAG
