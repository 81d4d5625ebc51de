#!/bin/bash
# rocprofv3 kernel trace of the default bench (native on one GPU) into gpurun_out/$1/prof
TAG=$1; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG && cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 3 "$@" > $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof.log 2>&1
