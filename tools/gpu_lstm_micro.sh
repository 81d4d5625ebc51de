#!/bin/bash
TAG=$1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG && \
timeout -k 10 120 python tools/lstm_layer_micro.py > gpurun_out/$TAG/micro64.log 2>&1 && \
IN=20 timeout -k 10 120 python tools/lstm_layer_micro.py > gpurun_out/$TAG/micro20.log 2>&1
