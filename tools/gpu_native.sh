#!/bin/bash
# native executor: tests, GPU-only replay times, bench eager vs --native
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/nat && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_model.py -k "native" > gpurun_out/nat/test.log 2>&1 && \
timeout -k 10 300 python tools/native_info.py 3 4 > gpurun_out/nat/info.log 2>&1 && \
timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/nat/eager.json 2> gpurun_out/nat/eager.err && \
timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --native > gpurun_out/nat/native4.json 2> gpurun_out/nat/native4.err && \
timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --native --streams 3 > gpurun_out/nat/native3.json 2> gpurun_out/nat/native3.err && \
timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --native --overlap-fe > gpurun_out/nat/native4o.json 2> gpurun_out/nat/native4o.err
