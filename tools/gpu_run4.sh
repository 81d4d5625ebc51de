#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest "tests/test_gpu_parity_s256.py::test_s256_training_trajectory_vs_reference" -m gpu -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/pytest_traj.log 2>&1 ; rc=$? ; \
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ; \
timeout -k 10 300 python bench.py --workload c4 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err && \
timeout -k 10 300 python bench.py --workload c4 --mode eager --no-cpu-baseline > gpurun_out/bench_c4_eager.json 2> gpurun_out/bench_c4_eager.err && \
timeout -k 10 300 python bench.py --workload c5 --steps 20 --warmup 3 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err && \
bash tools/gpu_prof.sh
