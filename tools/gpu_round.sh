#!/bin/bash
# round-end GPU pass at this tree: the whole GPU suite, smoke, the default bench (c2), the c4 /
# c5 workloads, the data-parallel probe and the literal J=6 front-end line, then rocprofv3 (kernel trace + PMC passes,
# tools/gpu_prof.sh)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 ; rc=$? ; \
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ; \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && \
timeout -k 10 300 python bench.py --workload c4 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err && \
timeout -k 10 300 python bench.py --workload c5 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err && \
timeout -k 10 300 python bench.py --ddp-probe --no-cpu-baseline > gpurun_out/bench_ddp_probe.json 2> gpurun_out/bench_ddp_probe.err && \
timeout -k 10 300 python bench.py --frontend j6 --no-cpu-baseline > gpurun_out/bench_j6.json 2> gpurun_out/bench_j6.err && \
bash tools/gpu_prof.sh
