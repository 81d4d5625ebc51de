#!/bin/bash
# rocprofv3 evidence for the c4 and c5 bench lines: kernel trace + stats of
# each workload (timed steps cut out by tools/step_stats.py between bench.py's markers), and for
# c5 the FETCH_SIZE / WRITE_SIZE passes of its roofline kernel k_scat_mod_spec.  Raw output under
# gpurun_out/prof_c4, prof_c5, pmc_c5; the summaries are copied into profiles/ by hand.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c4 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4 --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_c4.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_c5.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmc_c5 -o fetch --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc_c5_fetch.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmc_c5 -o write --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc_c5_write.log 2>&1
