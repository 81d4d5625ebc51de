#!/bin/bash
# ResidualMLP backward block-shape change: its tests, the step goldens, then a same-box bench A/B
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_resmlp_bf16.py tests/test_gpu_model.py tests/test_gpu_parity_s256.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/occ_tests.log 2>&1; rc=$?
if [ $rc -gt 1 ]; then exit $rc; fi
for i in 1 2; do
  for o in 1 0; do
    VAETEB_MLPB_OCC=$o timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/occ_b${o}_$i.json 2>/dev/null || exit 3
  done
done
