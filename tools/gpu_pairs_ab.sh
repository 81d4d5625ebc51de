#!/bin/bash
# full-step A/B of the pair kernel variant (VAETEB_PAIRS_DIRECT 0 = LDS-staged product, 1 = direct columns)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
for m in 0 1 0 1; do
  VAETEB_PAIRS_DIRECT=$m timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/p_$m.json 2> gpurun_out/p_$m.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/p_$m.json'));print('direct=$m',d['ms_per_step'],d['roofline']['avg_launch_ms'])"
done
