#!/bin/bash
# GPU round check: parity tests, eager + graph bench (no rebuild: the in-tree .so travels).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_eager.json 2> gpurun_out/bench_eager.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph > gpurun_out/bench_graph.json 2> gpurun_out/bench_graph.err
