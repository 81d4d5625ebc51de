cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06e
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06e/pytest_gpu.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest -x -s -q -p no:cacheprovider --timeout 240 --timeout-method thread tests/test_gpu_classifier.py -k "bench_precision" > gpurun_out/r06e/c4prec.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_prof_c45.sh || exit $?
timeout -k 10 120 python -X faulthandler tools/capture_probe.py model_lstm_info > gpurun_out/r06e/cap_lstm_info.log 2>&1 || exit $?
timeout -k 10 120 python -X faulthandler tools/capture_probe.py model_head_info > gpurun_out/r06e/cap_head_info.log 2>&1
echo "head_info rc=$?" >> gpurun_out/r06e/cap_head_info.log
