#!/bin/bash
# run-to-run spread of the default bench (3 runs)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_n$i.json 2> gpurun_out/bench_n$i.err || exit $?
done
