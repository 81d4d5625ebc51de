#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
for s in 1 2 3; do
  VAETEB_GRAD_SIDE_STREAM=$s timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_gs$s.json 2> gpurun_out/bench_gs$s.err || exit $?
done
