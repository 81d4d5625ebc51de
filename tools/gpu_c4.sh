#!/bin/bash
# config 4 bench + rocprofv3 kernel stats, and the c2 bench as a regression check
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c4 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4 --steps 3 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_c4.log 2>&1
