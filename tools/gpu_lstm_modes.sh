#!/bin/bash
# LSTM fused-projection placement modes: diagnostic + layer micro per mode, then bench per mode
TAG=$1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG || exit 1
for fm in 0 1 2; do
  VAETEB_LSTM_FWD_MODE=$fm VAETEB_LSTM_BWD_MODE=$((fm == 0 ? 1 : fm)) timeout -k 10 120 python tools/lstm_layer_micro.py > gpurun_out/$TAG/micro_m$fm.log 2>&1 || exit 1
done
VAETEB_LSTM_FWD_MODE=2 VAETEB_LSTM_BWD_MODE=2 timeout -k 10 120 python tools/diag_lstmx.py > gpurun_out/$TAG/diag_m2.log 2>&1 || exit 1
for fm in 0 2; do for bm in 1 2; do
  VAETEB_LSTM_FWD_MODE=$fm VAETEB_LSTM_BWD_MODE=$bm timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/$TAG/bench_f${fm}b${bm}.json 2> gpurun_out/$TAG/bench_f${fm}b${bm}.err || exit 1
done; done
