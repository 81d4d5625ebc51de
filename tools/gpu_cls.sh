#!/bin/bash
# classifier (config 4) GPU tests
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_classifier.py -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_cls.log 2>&1
