#!/bin/bash
# the 16-bit LSTM in the step: the all-bf16 step vs the reference's autocast spread (both LSTM
# precisions), the LSTM16 parity tests, and the default bench with / without --lstm 16-mixed
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_lstm16.py "tests/test_gpu_parity_s256.py::test_s256_bf16_step_within_reference_autocast_spread" -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_l16step.log 2>&1 ; rc=$? ; \
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ; \
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_l32.json 2> gpurun_out/bench_l32.err && \
timeout -k 10 200 python bench.py --no-cpu-baseline --lstm 16-mixed > gpurun_out/bench_l16.json 2> gpurun_out/bench_l16.err && \
B=256 L16=1 timeout -k 10 120 python tools/lstm_layer_micro.py > gpurun_out/l16_micro.log 2>&1
