#!/bin/bash
# Round-2 baseline: GPU parity suite, default bench, kernel trace (per-dispatch CSV) of 3 steps.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r2 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r2/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r2/bench_default.json 2> gpurun_out/r2/bench_default.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r2/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r2/trace.log 2>&1
