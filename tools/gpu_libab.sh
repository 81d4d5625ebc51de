#!/bin/bash
# same-box A/B of two builds of the library: A = vae-teb_amd/vaeteb/_lib/libvaeteb_A.so, B = the tree's build
TAG=$1; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG || exit 1
A=$GRAFT_REPO_ROOT/vae-teb_amd/vaeteb/_lib/libvaeteb_A.so
for r in 1 2 3; do
  VAETEB_LIB=$A timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 "$@" > gpurun_out/$TAG/A$r.json 2> gpurun_out/$TAG/A$r.err || exit 1
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 "$@" > gpurun_out/$TAG/B$r.json 2> gpurun_out/$TAG/B$r.err || exit 1
done
