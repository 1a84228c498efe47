#!/bin/bash
# The headline (granule layout, contiguous pool) in fresh processes, the
# block order alternated: the table's choice vs RSAMD_BLOCK_XCD=1 (XCD remap).
# Usage (via gpurun): bash tools/gpu_order_ab_headline.sh TAG [REPS]
set -o pipefail
TAG=${1:?tag}
REPS=${2:-6}
mkdir -p gpurun_out
OUT=gpurun_out/order_ab_headline_$TAG.txt
: > "$OUT"
for i in $(seq 1 "$REPS"); do
  for xcd in table 1; do
    if [ "$xcd" = table ]; then unset RSAMD_BLOCK_XCD; else export RSAMD_BLOCK_XCD=$xcd; fi
    timeout -k 10 120 python3 bench.py --no-extras --no-live-pmc --steps 20 --warmup 3 \
        > /tmp/oa.json 2> /tmp/oa.err || { tail -20 /tmp/oa.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('/tmp/oa.json').read().strip().splitlines()[-1])
print(json.dumps({'rep': $i, 'order': '$xcd' if '$xcd' == 'table' else 'xcd_remap', 'frac': d['roofline']['frac']}))" >> "$OUT"
  done
done
unset RSAMD_BLOCK_XCD
cat "$OUT"
