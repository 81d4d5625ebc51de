#!/bin/bash
# 16-bit MFMA LSTM: parity tests vs the 16-bit model + torch fp64, then the layer micro-benchmark
# at 2 and 4 samples per workgroup (VAETEB_L16_NS), B=256 and B=4 (one workgroup: the pure
# per-step latency), and without the global stores (VAETEB_L16_DIAG=1)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_lstm16.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_l16.log 2>&1 ; rc=$? ; \
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ; \
: > gpurun_out/l16_micro.log && \
for ns in 2 4; do
  for b in 256 4; do
    for d in 0 1; do
      echo "ns $ns B $b diag $d" >> gpurun_out/l16_micro.log
      VAETEB_L16_NS=$ns VAETEB_L16_DIAG=$d B=$b L16=1 timeout -k 10 120 python tools/lstm_layer_micro.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/l16_micro.log || exit 1
    done
  done
done
