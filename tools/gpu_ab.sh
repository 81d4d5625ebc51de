#!/bin/bash
# Same-box A/B of the training step: bench.py (no CPU baseline) alternating between two
# environment settings, N rounds each, then one rocprofv3 kernel-stats pass of setting B.
#   bash tools/gpu_ab.sh TAG "ENV_A" "ENV_B" [rounds] [extra bench args]
TAG=$1; A=$2; B=$3; N=${4:-2}; EXTRA=$5
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG || exit 1
for i in $(seq 1 $N); do
  env $A timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 --warmup 5 $EXTRA > gpurun_out/$TAG/a$i.json 2> gpurun_out/$TAG/a$i.err || exit 1
  env $B timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 --warmup 5 $EXTRA > gpurun_out/$TAG/b$i.json 2> gpurun_out/$TAG/b$i.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && export $B && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 3 $EXTRA > $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof.log 2>&1
