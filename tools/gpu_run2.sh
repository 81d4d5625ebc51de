cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_s256.py tests/test_gpu_loop.py -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread -k "trajectory or loop or j6 or production" > gpurun_out/pytest_traj.log 2>&1 ; rc=$? ; \
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ; \
timeout -k 10 300 python bench.py --no-cpu-baseline --ddp-probe > gpurun_out/bench_ddp_probe.json 2> gpurun_out/bench_ddp_probe.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --ddp-probe --mode eager > gpurun_out/bench_ddp_probe_eager.json 2> gpurun_out/bench_ddp_probe_eager.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --ddp-probe --reduce-bf16 > gpurun_out/bench_ddp_probe_bf16.json 2> gpurun_out/bench_ddp_probe_bf16.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && \
bash tools/gpu_prof.sh
