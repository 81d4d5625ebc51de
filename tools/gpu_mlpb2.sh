#!/bin/bash
# bf16 MLP kernels: parity tests, backward phase timeline, micro-benchmark
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/mlpb2 && \
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_resmlp_bf16.py > gpurun_out/mlpb2/test.log 2>&1 && \
timeout -k 10 100 python tools/mlpb_phases.py pre64 > gpurun_out/mlpb2/ph.log 2>&1 && \
timeout -k 10 100 python tools/mlpb_phases.py src130 >> gpurun_out/mlpb2/ph.log 2>&1 && \
timeout -k 10 100 python tools/mlpb_phases.py mu33 >> gpurun_out/mlpb2/ph.log 2>&1
