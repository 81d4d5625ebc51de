#!/bin/bash
# the J=6 end-to-end test with each pair-kernel form (diagnostic print of the worst gradient),
# the fp16 MLP rounded-model test, then the pair-kernel forms side by side
# (tools/pairs_micro.py): HIP events, a rocprofv3 kernel trace and an SQ counter pass
out=$GRAFT_REPO_ROOT/gpurun_out/pp
cd $GRAFT_REPO_ROOT && mkdir -p $out || exit 1
for h in 1 0; do
VAETEB_PAIRS_HALF=$h timeout -k 10 300 python -u -m pytest tests/test_gpu_parity_s256.py::test_j6_config2_step_end_to_end_vs_oracle -s -v --tb=short -p no:cacheprovider --timeout 250 --timeout-method thread > $out/t_j6_half$h.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_resmlp_bf16.py -k "rounded_fp64" -v --tb=short -p no:cacheprovider --timeout 250 --timeout-method thread > $out/t_mlp.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python tools/pairs_micro.py > $out/micro.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/pairs_micro.py > $out/prof.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace -d $out/pmc -o sq --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/pairs_micro.py > $out/pmc_sq.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM --kernel-trace -d $out/pmc -o inst --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/pairs_micro.py > $out/pmc_inst.log 2>&1
