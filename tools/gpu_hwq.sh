#!/bin/bash
# step time vs the number of HIP hardware queues per process (streams beyond it share queues and serialise)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_hwq$q.json 2> gpurun_out/bench_hwq$q.err || exit $?
done
