#!/bin/bash
# SQ counters of the bf16 conv weight-gradient kernel on decoder layer 2 (separate --pmc passes)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
  tag=$(echo $pmc | cut -c1-12 | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc $pmc -d $GRAFT_REPO_ROOT/gpurun_out/dwpmc_$tag -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/dw_micro.py 2 > $GRAFT_REPO_ROOT/gpurun_out/dwpmc_$tag.log 2>&1 || exit $?
done
