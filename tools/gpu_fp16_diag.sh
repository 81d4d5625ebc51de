#!/bin/bash
# fp16 diagnostics: per-stack KL deviations, the fp16 rounded-model tests of the MLP / conv kernels,
# the fp16 step tests, the classifier bench-precision test.  Usage: tools/gpu_fp16_diag.sh OUTDIR
out=$GRAFT_REPO_ROOT/gpurun_out/$1
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
timeout -k 10 300 python -u tools/fp16_diag2.py > $out/fp16_diag2.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -s -v -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_resmlp_bf16.py tests/test_gpu_conv_bf16.py tests/test_gpu_fp16.py "tests/test_gpu_classifier.py::test_seqvae_classifier_bench_precision_within_reference_16bit_spread" > $out/pytest_fp16.log 2>&1
exit 0
