#!/bin/bash
# Front-end parity tests, front-end micro-benchmark, default bench.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontend.py tests/test_gpu_api.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_fe.log 2>&1 && \
timeout -k 10 120 python tools/fe_micro.py > gpurun_out/fe_micro.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_fe.json 2> gpurun_out/bench_fe.err
