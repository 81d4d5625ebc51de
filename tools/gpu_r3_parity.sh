#!/bin/bash
# S=256 / bf16 / J6 parity tests (tests/test_gpu_parity_s256.py)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity_s256.py -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1
