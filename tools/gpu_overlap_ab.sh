#!/bin/bash
# step-level overlap options at this tree (same box, interleaved): default, --overlap-adam 1,
# --fe-in-graph 1, --overlap-fe
out=$GRAFT_REPO_ROOT/gpurun_out/ovl
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/b_def_$i.json 2> $out/b_def_$i.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --overlap-adam 1 > $out/b_oa_$i.json 2> $out/b_oa_$i.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --fe-in-graph 1 > $out/b_fig_$i.json 2> $out/b_fig_$i.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --overlap-fe > $out/b_ofe_$i.json 2> $out/b_ofe_$i.err || exit $?
done
