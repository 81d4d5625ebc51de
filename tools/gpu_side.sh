#!/bin/bash
# step time vs the number of side streams the model forks onto
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
for n in 2 3 4; do
  VAETEB_MAX_SIDE_STREAMS=$n timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_side$n.json 2> gpurun_out/bench_side$n.err || exit $?
done
