#!/bin/bash
# column sums with pinned arithmetic: bits vs the committed kernel (B = 2 and the bench's 256);
# deferred head weight gradients: bitwise test + A/B bench; then the timed-step profile + PMC
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab && rm -rf gpurun_out/prof gpurun_out/pmc && \
timeout -k 10 120 python tools/bisect_bits.py > gpurun_out/bis13.log 2>&1 && \
VAETEB_LIB=$GRAFT_REPO_ROOT/tools/probe/bis/lib_old.so timeout -k 10 120 python tools/bisect_bits.py >> gpurun_out/bis13.log 2>&1 && \
BISECT_B=256 timeout -k 10 120 python tools/bisect_bits.py >> gpurun_out/bis13.log 2>&1 && \
BISECT_B=256 VAETEB_LIB=$GRAFT_REPO_ROOT/tools/probe/bis/lib_old.so timeout -k 10 120 python tools/bisect_bits.py >> gpurun_out/bis13.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_model.py tests/test_gpu_lstm16.py -k "deferred or native_executor_bitwise or graph_capture or pair" > gpurun_out/pytest_defer.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/ab/d0.json 2> gpurun_out/ab/d0.err && \
VAETEB_HEAD_DW_DEFER=1 timeout -k 10 300 python bench.py > gpurun_out/ab/d1.json 2> gpurun_out/ab/d1.err && \
timeout -k 10 300 python bench.py > gpurun_out/ab/d0b.json 2> gpurun_out/ab/d0b.err && \
VAETEB_HEAD_DW_DEFER=1 timeout -k 10 300 python bench.py > gpurun_out/ab/d1b.json 2> gpurun_out/ab/d1b.err && \
bash tools/gpu_prof.sh
