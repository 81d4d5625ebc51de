#!/bin/bash
# Wide-row LayerNorm check: LN / model parity tests, bench, kernel stats.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_resmlp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_ln.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_ln.json 2> gpurun_out/bench_ln.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/profln -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/profln.log 2>&1
