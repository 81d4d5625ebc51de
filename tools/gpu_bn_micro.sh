#!/bin/bash
# BatchNorm backward column partials: block count / loads-in-flight settings (tools/bn_micro.py)
out=$GRAFT_REPO_ROOT/gpurun_out/bnm
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
timeout -k 10 120 python tools/bn_micro.py > $out/def.txt 2>&1 || exit $?
VAETEB_BN_BLOCKS=1024 timeout -k 10 120 python tools/bn_micro.py > $out/b1024.txt 2>&1 || exit $?
VAETEB_BN_BLOCKS=2048 timeout -k 10 120 python tools/bn_micro.py > $out/b2048.txt 2>&1 || exit $?
VAETEB_COLP_U=8 timeout -k 10 120 python tools/bn_micro.py > $out/u8.txt 2>&1 || exit $?
VAETEB_BN_BLOCKS=1024 VAETEB_COLP_U=8 timeout -k 10 120 python tools/bn_micro.py > $out/b1024u8.txt 2>&1 || exit $?
VAETEB_BN_FOLD=0 timeout -k 10 120 python tools/bn_micro.py > $out/nofold.txt 2>&1
