#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ntr && cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/ntr/t -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --native --steps 4 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/ntr/log 2>&1
