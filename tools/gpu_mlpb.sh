#!/bin/bash
# bf16 ResidualMLP kernels: parity tests, then the unchanged fp32 MLP tests
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/mlpb && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_resmlp_bf16.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/mlpb/pytest.log 2>&1
