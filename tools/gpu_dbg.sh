#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && timeout -k 10 200 python -u tools/debug_j6.py > gpurun_out/debug_j6.log 2>&1
