#!/bin/bash
# Kernel + HIP API trace of the bench: host enqueue time vs kernel start (host lag).
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d $GRAFT_REPO_ROOT/gpurun_out/profhip -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/profhip.log 2>&1
