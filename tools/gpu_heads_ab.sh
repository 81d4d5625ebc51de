#!/bin/bash
# Same-box A/B of the decoder-head GEMMs (tools/heads_micro.py) between a saved library
# (vae-teb_amd/vaeteb/_lib/ab/libvaeteb_old.so) and the current one.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/heads && \
for i in 1 2; do
  timeout -k 10 120 env VAETEB_LIB=$GRAFT_REPO_ROOT/vae-teb_amd/vaeteb/_lib/ab/libvaeteb_old.so python tools/heads_micro.py >> gpurun_out/heads/old.jsonl 2>> gpurun_out/heads/err.log || exit $?
  timeout -k 10 120 python tools/heads_micro.py >> gpurun_out/heads/new.jsonl 2>> gpurun_out/heads/err.log || exit $?
done
