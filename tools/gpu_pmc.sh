# HBM traffic of the roofline kernel: separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE)
cd $GRAFT_REPO_ROOT && python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 && cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmc -o fetch --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmc -o write --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc_write.log 2>&1
