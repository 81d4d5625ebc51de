#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 200 python tools/mlp_micro.py > gpurun_out/micro.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"; do
  tag=$(echo $pmc | cut -c1-12 | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc $pmc -d $GRAFT_REPO_ROOT/gpurun_out/pmc_$tag -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/mlp_micro.py mu33 > $GRAFT_REPO_ROOT/gpurun_out/pmc_$tag.log 2>&1 || exit $?
done
