#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_determinism.py "tests/test_gpu_parity_s256.py::test_s256_training_trajectory_vs_reference" -m gpu -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/pytest_det.log 2>&1 ; rc=$? ; \
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ; \
bash tools/gpu_capture_probe.sh
