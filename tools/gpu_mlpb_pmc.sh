#!/bin/bash
# bf16 MLP micro-benchmark + SQ counters of its kernels
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/mlpbp && \
timeout -k 10 120 python tools/mlpb_micro.py > gpurun_out/mlpbp/micro.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $GRAFT_REPO_ROOT/gpurun_out/mlpbp/p1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/mlpb_micro.py src130,pre64,mu33 --bf16-only > $GRAFT_REPO_ROOT/gpurun_out/mlpbp/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA -d $GRAFT_REPO_ROOT/gpurun_out/mlpbp/p2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/mlpb_micro.py src130,pre64,mu33 --bf16-only > $GRAFT_REPO_ROOT/gpurun_out/mlpbp/p2.log 2>&1
