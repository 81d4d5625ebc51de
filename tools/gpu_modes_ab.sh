#!/bin/bash
# same-box A/B of bench modes: default eager vs --prefetch (next batch's front-end one step ahead)
TAG=$1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG || exit 1
for r in 1 2 3; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/$TAG/eager_r$r.json 2> gpurun_out/$TAG/eager_r$r.err || exit 1
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --warmup 5 --prefetch > gpurun_out/$TAG/prefetch_r$r.json 2> gpurun_out/$TAG/prefetch_r$r.err || exit 1
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --warmup 5 --overlap-update > gpurun_out/$TAG/ovup_r$r.json 2> gpurun_out/$TAG/ovup_r$r.err || exit 1
done
