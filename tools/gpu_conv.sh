#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_bf16.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1
rc=$?; echo "conv rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_model.log 2>&1
rc=$?; echo "model rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_eager.json 2> gpurun_out/bench_eager.err || exit $?
bash tools/gpu_prof.sh
