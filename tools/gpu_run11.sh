#!/bin/bash
# the capture-end crash with a single-node capture tail: the head / both weight-gradient
# branches under capture, then the capture tests and an A/B bench with the branches kept
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab && rm -f gpurun_out/capprobe/summary.txt && \
PROBE_VARIANTS="model_head model_branches" bash tools/gpu_capture_probe.sh && \
grep -q "model_branches rc=0" gpurun_out/capprobe/summary.txt && \
VAETEB_CAPTURE_BRANCHES=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_model.py -k "graph or capture or native" > gpurun_out/pytest_branches.log 2>&1 && \
VAETEB_CAPTURE_BRANCHES=1 timeout -k 10 300 python bench.py > gpurun_out/ab/br1.json 2> gpurun_out/ab/br1.err && \
timeout -k 10 300 python bench.py > gpurun_out/ab/br0.json 2> gpurun_out/ab/br0.err && \
VAETEB_CAPTURE_BRANCHES=1 timeout -k 10 300 python bench.py > gpurun_out/ab/br1b.json 2> gpurun_out/ab/br1b.err && \
timeout -k 10 300 python bench.py > gpurun_out/ab/br0b.json 2> gpurun_out/ab/br0b.err
