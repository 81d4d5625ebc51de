#!/bin/bash
# Round-3 start: where the step's copies come from, eager vs native bench at the round-2 tree.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u tools/copy_sources.py > gpurun_out/copy_sources.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench_eager.json 2> gpurun_out/bench_eager.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --native > gpurun_out/bench_native.json 2> gpurun_out/bench_native.err
