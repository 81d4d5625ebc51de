#!/bin/bash
# same-box A/B of the ResidualMLP backward block shape (VAETEB_MLPB_OCC 1 / 2): kernel span
# and per-workgroup time from the phase stamps (tools/mlpb_phases.py), alternating twice
mkdir -p gpurun_out
for o in 1 2 1 2; do  # 2: the 32-wide stacks; 3: also 64-wide
  for s in pre64 scat43 dec50 mu33; do
    VAETEB_MLPB_OCC=$o timeout -k 10 120 python tools/mlpb_phases.py $s > gpurun_out/mlpb_tmp.log 2>&1 || exit 3
    echo "occ $o $(grep workgroups gpurun_out/mlpb_tmp.log)" >> gpurun_out/mlpb_ab.log
  done
done
