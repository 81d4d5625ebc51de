#!/bin/bash
# classifier (config 4), eval-mode and Lightning-mirror GPU tests
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_classifier.py tests/test_gpu_lightning.py -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_cls.log 2>&1
