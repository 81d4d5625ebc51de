#!/bin/bash
# round-3 GPU tests: parity (J6), SyncBN + multi-process fit; then the conv-block micro-benchmark
# with channel-lane staging (default) and the octet staging (VAETEB_CONV_CL=0)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/cm2 gpurun_out/cm3 && \
timeout -k 10 900 python -u -m pytest "tests/test_gpu_parity_s256.py::test_j6_config2_step_end_to_end_vs_oracle" tests/test_gpu_syncbn.py tests/test_gpu_conv_bf16.py -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/pytest_r3c.log 2>&1 ; rc=$? ; \
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ; \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/cm2/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/conv_micro.py > $GRAFT_REPO_ROOT/gpurun_out/cm2/log.txt 2>&1 && \
VAETEB_CONV_CL=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/cm3/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/conv_micro.py > $GRAFT_REPO_ROOT/gpurun_out/cm3/log.txt 2>&1
