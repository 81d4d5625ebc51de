#!/bin/bash
# session-start check at this tree: the GPU suite, smoke and the default bench line
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06f
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06f/pytest_gpu.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06f/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r06f/bench_default.json 2> gpurun_out/r06f/bench_default.err
