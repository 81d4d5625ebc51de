#!/bin/bash
# Same-box A/B of environment settings on the default bench, interleaved (the round-6 pair-kernel,
# BatchNorm-finalise, overlap-option and GEMM-order comparisons of DESIGN.md §9 ran this way).
# Usage: tools/gpu_env_ab.sh OUTDIR "VAR=a" "VAR=b" ...   (two rounds of every setting)
out=$GRAFT_REPO_ROOT/gpurun_out/$1
shift
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
for i in 1 2; do
  k=0
  for setting in "$@"; do
    k=$((k + 1))
    env $setting timeout -k 10 300 python bench.py --no-cpu-baseline > $out/b_${k}_$i.json 2> $out/b_${k}_$i.err || exit $?
  done
done
