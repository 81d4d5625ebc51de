#!/bin/bash
# same-box A/B of the whole tree: _old/ (an earlier commit's worktree with its own build) vs the tree
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/oldab || exit 1
for r in 1 2 3; do
  (cd _old && timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --warmup 5) > gpurun_out/oldab/old_r$r.json 2> gpurun_out/oldab/old_r$r.err || exit 1
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/oldab/new_r$r.json 2> gpurun_out/oldab/new_r$r.err || exit 1
  (cd _old && timeout -k 10 200 python tools/gpu_bound_probe.py 4) > gpurun_out/oldab/probe_old_r$r.log 2>&1 || exit 1
  timeout -k 10 200 python tools/gpu_bound_probe.py 4 > gpurun_out/oldab/probe_new_r$r.log 2>&1 || exit 1
done
