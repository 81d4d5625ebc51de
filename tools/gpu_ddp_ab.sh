#!/bin/bash
# the segmented-replay DDP bit identity (2 ranks, gloo, one GPU) with the bucket joins covering
# the backward's base stream (three runs), the comm stream joined with every executor stream
# before each bucket's all-reduce (DIAG 1), then the whole DDP test file.  A test failure (rc 1) goes on to
# the next variant; anything else (crash, timeout) stops.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ddpab || exit 1
T="tests/test_gpu_ddp.py::test_segmented_native_replay_equals_eager_ddp_step"
run() {
  env "$1" timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu $T > gpurun_out/ddpab/$2.log 2>&1
  rc=$?
  echo "$2 rc=$rc $(grep -m1 -o 'AssertionError: .*' gpurun_out/ddpab/$2.log | cut -c1-160)" >> gpurun_out/ddpab/summary.txt
  [ $rc -eq 0 ] || [ $rc -eq 1 ]
}
rm -f gpurun_out/ddpab/summary.txt
run VAETEB_X=1 fix1 && run VAETEB_X=1 fix2 && run VAETEB_X=1 fix3 && run VAETEB_DDP_DIAG=1 join1 && \
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ddp.py > gpurun_out/ddpab/file.log 2>&1
cat gpurun_out/ddpab/summary.txt
