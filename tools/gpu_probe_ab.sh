#!/bin/bash
# full GPU test suite, then GPU-only step time (tools/gpu_bound_probe.py) of library A
# (vae-teb_amd/vaeteb/_lib/libvaeteb_A.so) vs the tree's build, interleaved, 3 rounds
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
for r in 1 2 3; do
  VAETEB_LIB=vae-teb_amd/vaeteb/_lib/libvaeteb_A.so timeout -k 10 200 python tools/gpu_bound_probe.py 4 > gpurun_out/probeA_$r.log 2>&1 || exit 1
  timeout -k 10 200 python tools/gpu_bound_probe.py 4 > gpurun_out/probeB_$r.log 2>&1 || exit 1
done
