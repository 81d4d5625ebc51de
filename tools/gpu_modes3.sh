#!/bin/bash
# step-level A/B: LSTM weight gradients inline vs on side streams 1/2/3; prefetch / overlap-update pipelines
TAG=$1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG || exit 1
run() { local name=$1; shift; timeout -k 10 240 env "$@" > gpurun_out/$TAG/$name.json 2> gpurun_out/$TAG/$name.err || exit 1; }
for r in 1 2; do
run inline$r python bench.py --no-cpu-baseline --steps 30
run side1_$r VAETEB_LSTM_GRAD_SIDE_STREAM=1 python bench.py --no-cpu-baseline --steps 30
run side2_$r VAETEB_LSTM_GRAD_SIDE_STREAM=2 python bench.py --no-cpu-baseline --steps 30
run side3_$r VAETEB_LSTM_GRAD_SIDE_STREAM=3 python bench.py --no-cpu-baseline --steps 30
done
run ovu python bench.py --no-cpu-baseline --steps 30 --overlap-update
run pre python bench.py --no-cpu-baseline --steps 30 --prefetch
run nat python bench.py --no-cpu-baseline --steps 30 --native
