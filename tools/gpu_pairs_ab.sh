#!/bin/bash
# the tests that failed at the session start (MlpSpec.grad_pointers), the front-end tests, then the
# default bench with the half-image pair kernel (default) and the full-image one
# (VAETEB_PAIRS_HALF=0), interleaved on one box
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pab
T="tests/test_gpu_classifier.py::test_seqvae_classifier_vs_reference_golden tests/test_gpu_classifier.py::test_seqvae_classifier_bench_precision_within_reference_16bit_spread tests/test_gpu_classifier.py::test_seqvae_classifier_native_executor tests/test_gpu_conv_bf16.py::test_model_bf16_convs_close_to_fp32 tests/test_gpu_frontend.py"
timeout -k 10 500 python -u -m pytest $T -v --tb=short -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pab/t.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/pab/b_half$i.json 2> gpurun_out/pab/b_half$i.err || exit $?
VAETEB_PAIRS_HALF=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/pab/b_full$i.json 2> gpurun_out/pab/b_full$i.err || exit $?
done
