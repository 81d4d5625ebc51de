#!/bin/bash
# which capture topology crashes hipStreamEndCapture.  One variant per
# process, the least likely to crash first; the script stops at the first crash (rules: no
# more GPU work in a call after a segfault / abort / timeout).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/capprobe
for v in ${PROBE_VARIANTS:-fork_join reuse_branch eager_then_fork external_wait model_branches unjoined}; do
  AMD_LOG_LEVEL=${PROBE_LOG:-0} timeout -k 10 120 python -X faulthandler tools/capture_probe.py $v > gpurun_out/capprobe/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc" >> gpurun_out/capprobe/summary.txt
  if [ $rc -ne 0 ]; then exit 0; fi
done
