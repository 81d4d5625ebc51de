#!/bin/bash
# full GPU suite, then host enqueue / GPU-only step time (gpu_bound_probe) and bench per env variant
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
T=$1; shift
for r in 1 2; do
  i=0
  for V in "$@"; do
    E=$V; [ "$V" = "-" ] && E=""
    timeout -k 10 200 env $E python tools/gpu_bound_probe.py 4 > gpurun_out/$T/probe_v${i}_r$r.log 2>&1 || exit 1
    timeout -k 10 240 env $E python bench.py --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/$T/bench_v${i}_r$r.json 2> gpurun_out/$T/bench_v${i}_r$r.err || exit 1
    i=$((i+1))
  done
done
