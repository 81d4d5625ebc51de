#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && timeout -k 10 300 python tools/copy_sources.py > gpurun_out/copies.log 2>&1
