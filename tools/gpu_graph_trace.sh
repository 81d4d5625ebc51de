#!/bin/bash
# kernel trace of the graph-replay bench (concurrency of replayed branches)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gtr && cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/gtr/t -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --graph --steps 4 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/gtr/log 2>&1
