#!/bin/bash
# Critical-path sensitivity of the training step (diagnostic): the default bench with
# one kernel family turned into a no-op at a time (VAETEB_ABLATE, vaeteb/_lib.py).
# The step time saved bounds what making that family faster can buy.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/abl && \
for cfg in base vt_lstm_layer_bwd_weight vt_conv1d_bwd_weight_bf16_dy16 vt_mfma_linear_bwd_weight \
           vt_lstm_layer_fwd_x,vt_lstm_layer_bwd_x vt_resmlp_bf16_bwd vt_conv1d_bwd_dx_bf16_bn,vt_conv1d_bwd_gpad_bf16_bn \
           vt_adamw_step_dev vt_fe_pairs vt_fe_wavelet vt_resmlp_bf16_fwd vt_conv1d_bn_fwd_bf16 ; do
  if [ $cfg = base ]; then ab=""; else ab=$cfg; fi
  VAETEB_ABLATE=$ab timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/abl/$cfg.json 2> gpurun_out/abl/$cfg.err || exit 1
done
