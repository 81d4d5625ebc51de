#!/bin/bash
# rocprofv3 kernel trace + stats of the bench (eager), 3 timed steps; no rebuild.
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
