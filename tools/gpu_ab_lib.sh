#!/bin/bash
# Same-box A/B of the current library against vae-teb_amd/vaeteb/_lib/ab/libvaeteb_base.so (a build
# with one source file at its previous revision): bit-identity of two bf16 training steps
# (tools/lib_bitwise.py at S = 64 and S = 256), then the default bench twice per build,
# interleaved.  Usage: tools/gpu_ab_lib.sh OUTDIR [extra pytest files ...]
out=$GRAFT_REPO_ROOT/gpurun_out/$1; shift
base=$GRAFT_REPO_ROOT/vae-teb_amd/vaeteb/_lib/ab/libvaeteb_base.so
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread "$@" > $out/pytest.log 2>&1 || exit $?
fi
for s in 64 256; do
  timeout -k 10 120 env LB_S=$s python tools/lib_bitwise.py run $out/new_s$s.json > $out/lb.log 2>&1 || exit $?
  timeout -k 10 120 env LB_S=$s VAETEB_LIB=$base python tools/lib_bitwise.py run $out/base_s$s.json >> $out/lb.log 2>&1 || exit $?
  python tools/lib_bitwise.py compare $out/new_s$s.json $out/base_s$s.json >> $out/bitwise.txt 2>&1
done
for i in 1 2; do
  timeout -k 10 300 env VAETEB_LIB=$base python bench.py --no-cpu-baseline > $out/bench_base_$i.json 2> $out/bench_base_$i.err || exit $?
  timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench_new_$i.json 2> $out/bench_new_$i.err || exit $?
done
