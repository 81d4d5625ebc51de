#!/bin/bash
# full GPU suite, bit-equality of the tree's library vs libvaeteb_A.so on the training step,
# then GPU-only step time A vs tree (interleaved, 2 rounds)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmix && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/qt.log 2>&1 && \
VAETEB_LIB=vae-teb_amd/vaeteb/_lib/libvaeteb_A.so timeout -k 10 120 python tools/lib_bitwise.py run gpurun_out/bwA.json > gpurun_out/bw.log 2>&1 && \
timeout -k 10 120 python tools/lib_bitwise.py run gpurun_out/bwB.json >> gpurun_out/bw.log 2>&1 || exit 1
python tools/lib_bitwise.py compare gpurun_out/bwA.json gpurun_out/bwB.json >> gpurun_out/bw.log 2>&1
for r in 1 2; do
  VAETEB_LIB=vae-teb_amd/vaeteb/_lib/libvaeteb_A.so timeout -k 10 200 python tools/gpu_bound_probe.py 4 > gpurun_out/pmix/A_$r.log 2>&1 || exit 1
  timeout -k 10 200 python tools/gpu_bound_probe.py 4 > gpurun_out/pmix/B_$r.log 2>&1 || exit 1
  echo "A r$r: $(grep GPU gpurun_out/pmix/A_$r.log | tail -1)" >> gpurun_out/pmix/summary.txt
  echo "B r$r: $(grep GPU gpurun_out/pmix/B_$r.log | tail -1)" >> gpurun_out/pmix/summary.txt
done
