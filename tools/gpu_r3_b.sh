#!/bin/bash
# parity tests (S=256 / bf16 / J6) and the isolated decoder conv-block kernel timings
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/cm && \
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity_s256.py -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1 ; rc=$? ; \
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ; \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/cm/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/conv_micro.py > $GRAFT_REPO_ROOT/gpurun_out/cm/log.txt 2>&1
