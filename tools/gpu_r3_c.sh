#!/bin/bash
# new round-3 GPU tests: parity (J6), SyncBN + multi-process fit
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest "tests/test_gpu_parity_s256.py::test_j6_config2_step_end_to_end_vs_oracle" tests/test_gpu_syncbn.py -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/pytest_r3c.log 2>&1
