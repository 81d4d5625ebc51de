#!/bin/bash
# same-box A/B of an environment switch: A = with "$2" (e.g. VAETEB_X=0), B = default; 3 rounds
TAG=$1; AENV=$2
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG || exit 1
for r in 1 2 3; do
  timeout -k 10 240 env $AENV python bench.py --no-cpu-baseline --steps 30 > gpurun_out/$TAG/A$r.json 2> gpurun_out/$TAG/A$r.err || exit 1
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/$TAG/B$r.json 2> gpurun_out/$TAG/B$r.err || exit 1
done
