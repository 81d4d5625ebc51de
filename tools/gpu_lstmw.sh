#!/bin/bash
# LSTM weight gradients in one pass: full GPU tests, then A/B bench
TAG=$1; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || exit 1
run() {  # name, env..., -- bench args
    local name=$1; shift
    timeout -k 10 240 env "$@" > gpurun_out/$TAG/$name.json 2> gpurun_out/$TAG/$name.err || exit 1
}
run fused python bench.py --no-cpu-baseline --steps 30
run unfused VAETEB_LSTM_FUSED=0 python bench.py --no-cpu-baseline --steps 30
run fused2 python bench.py --no-cpu-baseline --steps 30
