#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_eager.json 2> gpurun_out/bench_eager.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph > gpurun_out/bench_graph.json 2> gpurun_out/bench_graph.err || exit $?
bash tools/gpu_prof.sh
