#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r2 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_lightning.py tests/test_gpu_model.py -k "ddp or graph or fit or eval" -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r2/pytest_fix.log 2>&1
