#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python tools/host_prof.py > gpurun_out/host_prof.log 2>&1 && \
VAETEB_LOCKSTEP=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_nols.json 2> gpurun_out/bench_nols.err && \
VAETEB_LOCKSTEP=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph > gpurun_out/bench_graph.json 2> gpurun_out/bench_graph.err
