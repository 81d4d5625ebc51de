#!/bin/bash
# Critical-path sensitivity of the training step (diagnostic): the default bench with
# one kernel family turned into a no-op at a time (VAETEB_ABLATE, vaeteb/_lib.py).
# The step time saved bounds what making that family faster can buy.  Also: the
# multi-GPU hardware-queue budget (main + 2 side streams) and the native executor on 1 GPU.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/abl && \
VAETEB_MAX_SIDE_STREAMS=2 VAETEB_GRAD_SIDE_STREAM=2 timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/abl/side2.json 2> gpurun_out/abl/side2.err && \
timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --native > gpurun_out/abl/native.json 2> gpurun_out/abl/native.err && \
for cfg in base vt_lstm_layer_bwd_weight vt_conv1d_bwd_weight_bf16_dy16 vt_mfma_linear_bwd_weight \
           vt_lstm_layer_fwd_x,vt_lstm_layer_bwd_x vt_resmlp_bf16_bwd vt_conv1d_bwd_dx_bf16_bn,vt_conv1d_bwd_gpad_bf16_bn \
           vt_adamw_step_dev vt_fe_pairs vt_fe_wavelet vt_resmlp_bf16_fwd vt_conv1d_bn_fwd_bf16 ; do
  if [ $cfg = base ]; then ab=""; else ab=$cfg; fi
  VAETEB_ABLATE=$ab timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/abl/$cfg.json 2> gpurun_out/abl/$cfg.err || exit 1
done
