#!/bin/bash
# production-geometry + parity tests, then the step ablations (tools/ablate_step.sh)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_s256.py "tests/test_gpu_frontend.py::test_frontend_vs_reference_golden" -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/pytest_r3e.log 2>&1 ; rc=$? ; \
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ; \
bash tools/ablate_step.sh
