#!/bin/bash
# Critical-path sensitivity of the training step (diagnostic): the default bench (native
# executor) with one kernel family turned into a no-op at a time (VAETEB_ABLATE, vaeteb/_lib.py).
# The step time saved bounds what making that family faster can buy; the results are wrong
# by construction (never a training setting).  Round 5: the entry points of the current step.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/abl && \
for cfg in base vt_fe_pairs vt_fe_wavelet vt_resmlp_bf16_bwd vt_resmlp_bf16_fwd vt_lstm16_pair_bwd \
           vt_lstm16_pair_fwd vt_batchnorm_bwd_coef,vt_batchnorm_bwd_x16 vt_conv1d_bwd_dx16 \
           vt_conv1d_bwd_weight_bf16_dy16s vt_conv1d_bn_fwd_bf16 \
           vt_mfma_linear_fwd,vt_mfma_linear_bwd_data,vt_mfma_linear_bwd_weight vt_adamw_step_dev_shadow \
           vt_lstm16_layer_bwd_weight ; do
  if [ $cfg = base ]; then ab=""; else ab=$cfg; fi
  VAETEB_ABLATE=$ab timeout -k 10 150 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/abl/$cfg.json 2> gpurun_out/abl/$cfg.err || exit 1
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abl/$cfg.json)"
done
