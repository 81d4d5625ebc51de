#!/bin/bash
# round-4 GPU pass: parity / trajectory / loop / shadow tests with their printed measurements,
# the rest of the GPU suite, smoke, the default bench, the DDP-probe benches, then rocprofv3.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity_s256.py tests/test_gpu_loop.py "tests/test_gpu_elbo_optim.py::test_adamw_writes_bf16_shadows_same_bits" -m gpu -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1 ; rc=$? ; \
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ; \
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread --deselect tests/test_gpu_parity_s256.py --deselect tests/test_gpu_loop.py > gpurun_out/pytest_gpu.log 2>&1 ; rc=$? ; \
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ; \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && \
VAETEB_SHADOW_UPDATE=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_noshadow.json 2> gpurun_out/bench_noshadow.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --ddp-probe > gpurun_out/bench_ddp_probe.json 2> gpurun_out/bench_ddp_probe.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --ddp-probe --mode eager > gpurun_out/bench_ddp_probe_eager.json 2> gpurun_out/bench_ddp_probe_eager.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --ddp-probe --reduce-bf16 > gpurun_out/bench_ddp_probe_bf16.json 2> gpurun_out/bench_ddp_probe_bf16.err && \
bash tools/gpu_prof.sh
