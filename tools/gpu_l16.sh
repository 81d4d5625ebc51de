#!/bin/bash
# 16-bit MFMA LSTM: parity tests vs the 16-bit model + torch fp64, error localisation
# (tools/diag_l16.py), the layer micro-benchmark (B=4: one workgroup, the pure per-step
# latency) and the in-kernel per-step segment stamps (tools/lstm16_stamps.py)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_lstm16.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_l16.log 2>&1 ; rc=$? ; \
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ; \
timeout -k 10 120 python tools/diag_l16.py > gpurun_out/diag_l16.log 2>&1 && \
L16=1 timeout -k 10 120 python tools/lstm_layer_micro.py > gpurun_out/l16_micro.log 2>&1 && \
B=4 L16=1 timeout -k 10 120 python tools/lstm_layer_micro.py >> gpurun_out/l16_micro.log 2>&1 && \
timeout -k 10 120 python tools/lstm16_stamps.py >> gpurun_out/l16_micro.log 2>&1 && \
B=256 timeout -k 10 120 python tools/lstm16_stamps.py >> gpurun_out/l16_micro.log 2>&1
