#!/bin/bash
# fused LSTM projections: LSTM / model GPU tests, then A/B benches (unfused, fused, fused + side-stream weight grads)
TAG=$1; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || exit 1
run() {  # name, env..., -- bench args
    local name=$1; shift
    timeout -k 10 240 env "$@" > gpurun_out/$TAG/$name.json 2> gpurun_out/$TAG/$name.err || exit 1
}
run unfused VAETEB_LSTM_FUSED=0 python bench.py --no-cpu-baseline --steps 30
run fused python bench.py --no-cpu-baseline --steps 30
run fused_side3 VAETEB_LSTM_GRAD_SIDE_STREAM=3 python bench.py --no-cpu-baseline --steps 30
run fused_side2 VAETEB_LSTM_GRAD_SIDE_STREAM=2 python bench.py --no-cpu-baseline --steps 30
run fused2 python bench.py --no-cpu-baseline --steps 30
