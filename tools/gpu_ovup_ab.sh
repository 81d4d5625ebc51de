#!/bin/bash
# same-box A/B: default eager step vs --overlap-update (next batch's front-end beside clip + AdamW)
T=$1; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$T || exit 1
for r in 1 2 3; do
  timeout -k 10 240 env "$@" python bench.py --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/$T/eager_r$r.json 2> gpurun_out/$T/eager_r$r.err || exit 1
  timeout -k 10 240 env "$@" python bench.py --no-cpu-baseline --steps 30 --warmup 5 --overlap-update > gpurun_out/$T/ovup_r$r.json 2> gpurun_out/$T/ovup_r$r.err || exit 1
done
