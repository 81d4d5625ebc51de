#!/bin/bash
# default bench + GPU-only step time + a GPU-bound kernel trace (tools/critchain.py input)
# usage: gpu_step_probe.sh TAG
TAG=$1; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err && \
timeout -k 10 300 python tools/gpu_bound_probe.py 4 > gpurun_out/$TAG/probe.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/gbt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/gpu_bound_probe.py 2 > $GRAFT_REPO_ROOT/gpurun_out/$TAG/gbt.log 2>&1
