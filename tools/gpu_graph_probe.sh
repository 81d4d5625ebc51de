#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gp && \
timeout -k 10 200 python -u tools/graph_probe.py --heads bf16 --conv bf16 --serial > gpurun_out/gp/bb_serial.log 2>&1 && \
VAETEB_HEAD_GRAD_SIDE_STREAM=0 timeout -k 10 200 python -u tools/graph_probe.py --heads bf16 --conv bf16 > gpurun_out/gp/bb_noside.log 2>&1
