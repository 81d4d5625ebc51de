#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_resmlp.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_mlp.log 2>&1
rc=$?; echo "mlp rc=$rc"; [ $rc -le 1 ] || exit $rc
bash tools/gpu_prof.sh
