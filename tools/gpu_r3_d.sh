#!/bin/bash
# round-3 GPU tests touched this session
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity_s256.py tests/test_gpu_syncbn.py tests/test_gpu_conv_bf16.py tests/test_gpu_resmlp_bf16.py "tests/test_gpu_model.py::test_measure_transfer_entropy_vs_reference_golden" "tests/test_gpu_model.py::test_lstm_fused_chunk_handoff_bitwise_fresh_process" tests/test_gpu_ddp.py -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/pytest_r3d.log 2>&1
