#!/bin/bash
# step time vs the side stream of the LSTM weight gradients (0 = inline)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_perf.log 2>&1 && \
for s in 0 2 3; do
  VAETEB_LSTM_GRAD_SIDE_STREAM=$s timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_ls$s.json 2> gpurun_out/bench_ls$s.err || exit $?
done
