#!/bin/bash
# GPU-only step time (gpu_bound_probe, 4 steps) per env variant ("-" = defaults), interleaved rounds
T=$1; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$T || exit 1
for r in 1 2; do
  i=0
  for V in "$@"; do
    E=$V; [ "$V" = "-" ] && E=""
    timeout -k 10 200 env $E python tools/gpu_bound_probe.py 4 > gpurun_out/$T/v${i}_r$r.log 2>&1 || exit 1
    echo "v$i ($V) r$r: $(grep GPU gpurun_out/$T/v${i}_r$r.log | tail -1)" >> gpurun_out/$T/summary.txt
    i=$((i+1))
  done
done
