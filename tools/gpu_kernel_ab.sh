#!/bin/bash
# same-box A/B of one kernel-selection variable: tools/gpu_kernel_ab.sh VAR V0 V1 -> the default
# bench under rocprofv3 --kernel-trace --stats (csv) for VAR=V0, V1, V0, V1 in gpurun_out/kab_<V>_<i>/
cd /tmp && export TMPDIR=/tmp
i=0
for v in $2 $3 $2 $3; do
  i=$((i + 1))
  export $1=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/kab_${v}_$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/kab_${v}_$i.json 2> $GRAFT_REPO_ROOT/gpurun_out/kab_${v}_$i.err || exit 3
done
