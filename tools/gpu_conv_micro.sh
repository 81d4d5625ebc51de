#!/bin/bash
TAG=$1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG && cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/conv_micro.py > $GRAFT_REPO_ROOT/gpurun_out/$TAG/log.txt 2>&1
