#!/bin/bash
# same-box A/B/... of environment switches: each argument after the tag is one variant
# ("-" = defaults), benched in interleaved rounds; prints ms_per_step per variant and round.
TAG=$1; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG || exit 1
for r in 1 2; do
  i=0
  for V in "$@"; do
    E=$V; [ "$V" = "-" ] && E=""
    timeout -k 10 240 env $E python bench.py --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/$TAG/v${i}_r$r.json 2> gpurun_out/$TAG/v${i}_r$r.err || exit 1
    echo "variant $i ($V) round $r: $(python -c "import json;print(json.load(open('gpurun_out/$TAG/v${i}_r$r.json'))['ms_per_step'])")" | tee -a gpurun_out/$TAG/summary.txt
    i=$((i+1))
  done
done
