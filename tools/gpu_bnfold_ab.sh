#!/bin/bash
# BatchNorm column-sum finalize in the partial kernel (default) vs the separate k_bn_finalize launch
# (VAETEB_BN_FOLD=0), interleaved on one box
out=$GRAFT_REPO_ROOT/gpurun_out/bnf
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
for i in 1 2 3; do
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/b_f1_$i.json 2> $out/b_f1_$i.err || exit $?
VAETEB_BN_FOLD=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $out/b_f0_$i.json 2> $out/b_f0_$i.err || exit $?
done
