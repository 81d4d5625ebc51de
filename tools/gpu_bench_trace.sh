#!/bin/bash
# default bench (and an A/B leg with extra args), then a per-dispatch kernel trace of 3 steps
# usage: gpu_bench_trace.sh TAG [extra bench args for the A/B leg]
TAG=$1; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 "$@" > gpurun_out/$TAG/bench_ab.json 2> gpurun_out/$TAG/bench_ab.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/$TAG/trace.log 2>&1
