#!/bin/bash
# trajectory + determinism at the reverted column sums, then the capture probes
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_parity_s256.py -k trajectory tests/test_gpu_determinism.py > gpurun_out/pytest_traj9.log 2>&1 && \
rm -f gpurun_out/capprobe/summary.txt && \
PROBE_VARIANTS="unjoined_refork model_head_join model_head" bash tools/gpu_capture_probe.sh
