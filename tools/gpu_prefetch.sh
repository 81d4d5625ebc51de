#!/bin/bash
# eager step vs the two front-end overlap variants (next batch's front-end on the model's side streams)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --overlap-update > gpurun_out/bench_ou.json 2> gpurun_out/bench_ou.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --prefetch > gpurun_out/bench_pf.json 2> gpurun_out/bench_pf.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_nopf.json 2> gpurun_out/bench_nopf.err
