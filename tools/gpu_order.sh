#!/bin/bash
# A/B of the lockstep node-creation order (VAETEB_LOCKSTEP_MAIN_FIRST none / enc / all)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
for m in none enc all none enc all; do
  VAETEB_LOCKSTEP_MAIN_FIRST=$m timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/o_$m.json 2> gpurun_out/o_$m.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/o_$m.json'));print('$m',d['ms_per_step'],d['host_enqueue_ms_per_step'])"
done
