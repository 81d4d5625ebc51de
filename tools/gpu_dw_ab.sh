#!/bin/bash
# conv parity tests, conv dW micro-benchmark A (libvaeteb_A.so) vs tree, GPU-only step time A vs tree
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_bf16.py tests/test_gpu_model.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/qt.log 2>&1 && \
VAETEB_LIB=vae-teb_amd/vaeteb/_lib/libvaeteb_A.so timeout -k 10 120 python tools/dw_micro.py > gpurun_out/dwA.log 2>&1 && \
timeout -k 10 120 python tools/dw_micro.py > gpurun_out/dwB.log 2>&1 && \
for r in 1 2; do
  VAETEB_LIB=vae-teb_amd/vaeteb/_lib/libvaeteb_A.so timeout -k 10 200 python tools/gpu_bound_probe.py 4 > gpurun_out/probeA_$r.log 2>&1 || exit 1
  timeout -k 10 200 python tools/gpu_bound_probe.py 4 > gpurun_out/probeB_$r.log 2>&1 || exit 1
done
