#!/bin/bash
# same-box A/B of the BN-backward bf16 row kernel (VAETEB_BNX16_PF 0 / 1), tools/bn_micro.py
mkdir -p gpurun_out
for v in 0 1 0 1; do
  echo "== PF $v" >> gpurun_out/bn_ab.log
  VAETEB_BNX16_PF=$v timeout -k 10 120 python tools/bn_micro.py >> gpurun_out/bn_ab.log 2>&1 || exit 3
done
