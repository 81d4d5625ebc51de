#!/bin/bash
# GPU check at the current tree: the parity / trajectory / bench-size tests with their printed
# measurements (-s), then the whole GPU suite, smoke and the default bench.
#   tools/gpu_check.sh [extra pytest node ids for the -s pass]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity_s256.py tests/test_gpu_loop.py "$@" -m gpu -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1 ; rc=$? ; \
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ; \
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread --deselect tests/test_gpu_parity_s256.py --deselect tests/test_gpu_loop.py > gpurun_out/pytest_gpu.log 2>&1 ; rc=$? ; \
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ; \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
