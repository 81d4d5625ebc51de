#!/bin/bash
# Same-box sweep of bench.py settings (native default mode): each setting run N times, interleaved.
#   bash tools/gpu_sweep.sh TAG N "label|ENV...|ARGS" ...
TAG=$1; N=$2; shift 2
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG || exit 1
for i in $(seq 1 $N); do
  k=0
  for spec in "$@"; do
    IFS='|' read -r label envs args <<< "$spec"
    env $envs timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 --warmup 5 $args > gpurun_out/$TAG/${label}_$i.json 2> gpurun_out/$TAG/${label}_$i.err || exit 1
  done
done
