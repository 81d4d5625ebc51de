#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 120 python tools/bisect_bits.py > gpurun_out/bis_cur.log 2>&1 && \
VAETEB_LIB=$GRAFT_REPO_ROOT/tools/probe/bis/lib_norm_old.so timeout -k 10 120 python tools/bisect_bits.py > gpurun_out/bis_norm.log 2>&1 && \
VAETEB_LIB=$GRAFT_REPO_ROOT/tools/probe/bis/lib_cbd_old.so timeout -k 10 120 python tools/bisect_bits.py > gpurun_out/bis_cbd.log 2>&1
