#!/bin/bash
# tests touched by the prepass / deferral / conv staging changes, then eager vs native benches
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_elbo_optim.py tests/test_gpu_conv_bf16.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/qt.log 2>&1 && \
bash tools/gpu_multi_ab.sh ab3 - VAETEB_PREPASS=0 && \
for r in 1 2; do timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --warmup 5 --native > gpurun_out/ab3/native_r$r.json 2> gpurun_out/ab3/native_r$r.err || exit 1; done
