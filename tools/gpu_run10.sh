#!/bin/bash
# LSTM layer pairs: bitwise + parity tests, A/B bench (pairs on / off / 4 samples per WG),
# then the head-branch capture crash with HIP API logging (the last step: it segfaults)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab && \
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_lstm16.py tests/test_gpu_model.py > gpurun_out/pytest_pair.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/ab/pair1.json 2> gpurun_out/ab/pair1.err && \
VAETEB_L16_PAIR=0 timeout -k 10 300 python bench.py > gpurun_out/ab/pair0.json 2> gpurun_out/ab/pair0.err && \
VAETEB_L16_PAIR_NS=4 timeout -k 10 300 python bench.py > gpurun_out/ab/pair1ns4.json 2> gpurun_out/ab/pair1ns4.err && \
timeout -k 10 300 python bench.py > gpurun_out/ab/pair1b.json 2> gpurun_out/ab/pair1b.err && \
VAETEB_L16_PAIR=0 timeout -k 10 300 python bench.py > gpurun_out/ab/pair0b.json 2> gpurun_out/ab/pair0b.err && \
mkdir -p gpurun_out/capprobe && \
AMD_LOG_LEVEL=3 timeout -k 10 120 python -X faulthandler tools/capture_probe.py model_head 2>&1 | tail -n 4000 > gpurun_out/capprobe/model_head_log3.txt
