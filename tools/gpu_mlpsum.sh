#!/bin/bash
# k_mlpb_sum with 64 loads in flight: ResidualMLP tests, two bench lines (ELBO must equal the
# previous tree's bit for bit), a kernel trace of the bench for the kernel's time
out=$GRAFT_REPO_ROOT/gpurun_out/mlpsum
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_resmlp_bf16.py -q --tb=short -p no:cacheprovider --timeout 200 --timeout-method thread > $out/t.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/b_$i.json 2> $out/b_$i.err || exit $?
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/prof.log 2>&1
