#!/bin/bash
# eager vs hipGraph step at the current tree (20 timed steps each)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/m_eager.json 2> gpurun_out/m_eager.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph > gpurun_out/m_graph.json 2> gpurun_out/m_graph.err && \
VAETEB_LOCKSTEP=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph > gpurun_out/m_graph_nols.json 2> gpurun_out/m_graph_nols.err
