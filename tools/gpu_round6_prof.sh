#!/bin/bash
# round-6 evidence, part 1: rocprofv3 of the default bench (kernel trace + stats, FETCH / WRITE /
# SQ passes: tools/gpu_prof.sh) and of the c4 / c5 workloads (tools/gpu_prof_c45.sh)
cd $GRAFT_REPO_ROOT && rm -rf gpurun_out/prof gpurun_out/pmc gpurun_out/prof_c4 gpurun_out/prof_c5 gpurun_out/pmc_c5 && \
bash tools/gpu_prof.sh && bash tools/gpu_prof_c45.sh
