#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_pf.json 2> gpurun_out/bench_pf.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-prefetch > gpurun_out/bench_nopf.json 2> gpurun_out/bench_nopf.err && \
timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c4pf.json 2> gpurun_out/bench_c4pf.err
