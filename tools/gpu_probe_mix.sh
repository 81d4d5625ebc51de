#!/bin/bash
# GPU-only step time: _old worktree vs the tree with env variants (interleaved, 2 rounds)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmix || exit 1
for r in 1 2; do
  (cd _old && timeout -k 10 200 python tools/gpu_bound_probe.py 4) > gpurun_out/pmix/old_r$r.log 2>&1 || exit 1
  echo "old r$r: $(grep GPU gpurun_out/pmix/old_r$r.log | tail -1)" >> gpurun_out/pmix/summary.txt
  i=0
  for V in "$@"; do
    E=$V; [ "$V" = "-" ] && E=""
    timeout -k 10 200 env $E python tools/gpu_bound_probe.py 4 > gpurun_out/pmix/v${i}_r$r.log 2>&1 || exit 1
    echo "v$i ($V) r$r: $(grep GPU gpurun_out/pmix/v${i}_r$r.log | tail -1)" >> gpurun_out/pmix/summary.txt
    i=$((i+1))
  done
done
