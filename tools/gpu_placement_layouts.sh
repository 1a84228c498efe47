#!/bin/bash
# Placement robustness of the headline batch (4+2 x 1 MiB x 4096 encode) per
# layout and allocator: every run is a fresh process with fresh allocations,
# the four cases interleaved, REPS rounds.  Usage (via gpurun):
#   bash tools/gpu_placement_layouts.sh TAG [REPS]
set -o pipefail
TAG=${1:?tag}
REPS=${2:-4}
mkdir -p gpurun_out
OUT=gpurun_out/placement_layouts_$TAG.txt
: > "$OUT"
for i in $(seq 1 "$REPS"); do
  for layout in ${LAYOUTS:-packed granule}; do
    for alloc in ${ALLOCS:-contiguous hipmalloc}; do
      echo "== rep $i layout $layout alloc $alloc $(date +%T)"
      timeout -k 10 120 python3 bench.py --no-extras --no-live-pmc --steps 20 --warmup 3 --layout $layout --alloc $alloc \
          > /tmp/pl.json 2> /tmp/pl.err || { tail -20 /tmp/pl.err; exit 1; }
      python3 -c "
import json,sys
d=json.loads(open('/tmp/pl.json').read().strip().splitlines()[-1])
print(json.dumps({'rep': $i, 'layout': '$layout', 'alloc': '$alloc', 'frac': d['roofline']['frac'], 'value': d['value'], 'hbm_alloc': d['config'].get('hbm_alloc'), 'hbm_layout': d['config'].get('hbm_layout')}))" >> "$OUT"
    done
  done
done
cat "$OUT"
