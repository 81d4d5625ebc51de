#!/bin/bash
# Quick check after a kernel change: LSTM + optimizer parity tests, the LSTM layer
# micro-benchmark, and the default bench (eager) at the current tree.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_elbo_optim.py tests/test_gpu_conv_bf16.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/qt.log 2>&1 && \
timeout -k 10 120 python tools/lstm_layer_micro.py > gpurun_out/lstm_micro.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err
