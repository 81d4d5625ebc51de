#!/bin/bash
# eager vs hipGraph replay of the training step (bf16 heads + convs), plus a kernel trace of the graph run
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ga && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/ga/eager.json 2> gpurun_out/ga/eager.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --graph > gpurun_out/ga/graph.json 2> gpurun_out/ga/graph.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/ga/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --no-cpu-baseline --graph > $GRAFT_REPO_ROOT/gpurun_out/ga/trace.log 2>&1
