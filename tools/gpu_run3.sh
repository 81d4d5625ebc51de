#!/bin/bash
# round-4 GPU pass 3: the tests changed since pass 2, the DDP-probe / c4 benches, then rocprofv3
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest "tests/test_gpu_parity_s256.py::test_s256_training_trajectory_vs_reference" tests/test_gpu_ddp.py "tests/test_gpu_classifier.py::test_seqvae_classifier_native_executor" "tests/test_gpu_frontend.py::test_pairs_persistent_kernel_bitwise" "tests/test_gpu_frontend.py::test_frontend_bench_batch_rows_equal_small_batch" -m gpu -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/pytest_r3.log 2>&1 ; rc=$? ; \
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ; \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --ddp-probe > gpurun_out/bench_ddp_probe.json 2> gpurun_out/bench_ddp_probe.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --ddp-probe --reduce-bf16 > gpurun_out/bench_ddp_probe_bf16.json 2> gpurun_out/bench_ddp_probe_bf16.err && \
timeout -k 10 300 python bench.py --workload c4 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err && \
timeout -k 10 300 python bench.py --workload c4 --mode eager --no-cpu-baseline > gpurun_out/bench_c4_eager.json 2> gpurun_out/bench_c4_eager.err && \
bash tools/gpu_prof.sh
