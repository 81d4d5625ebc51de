#!/bin/bash
# A/B of bench modes / tuning switches: one short bench per variant
TAG=$1; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG || exit 1
run() {  # name, env..., -- bench args
    local name=$1; shift
    timeout -k 10 240 env "$@" > gpurun_out/$TAG/$name.json 2> gpurun_out/$TAG/$name.err || exit 1
}
run default python bench.py --no-cpu-baseline --steps 30
run prefetch python bench.py --no-cpu-baseline --steps 30 --prefetch
run overlap python bench.py --no-cpu-baseline --steps 30 --overlap-update
run graph python bench.py --no-cpu-baseline --steps 30 --graph
run tpw1 VAETEB_MLPB_TPW=1 python bench.py --no-cpu-baseline --steps 30
run default2 python bench.py --no-cpu-baseline --steps 30
