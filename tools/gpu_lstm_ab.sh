#!/bin/bash
# LSTM kernels: fused-vs-plain row diagnostic, layer micro-benchmarks, model GPU tests, bench
TAG=$1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG && \
timeout -k 10 120 python tools/diag_lstmx.py > gpurun_out/$TAG/diag.log 2>&1 && \
timeout -k 10 120 python tools/lstm_layer_micro.py > gpurun_out/$TAG/micro64.log 2>&1 && \
IN=20 timeout -k 10 120 python tools/lstm_layer_micro.py > gpurun_out/$TAG/micro20.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 && \
timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err && \
timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/$TAG/bench2.json 2> gpurun_out/$TAG/bench2.err
