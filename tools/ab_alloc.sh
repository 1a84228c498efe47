#!/bin/bash
# A/B of the stripe pool's allocation (bench.py --alloc): physically
# contiguous (rs_dev_alloc) against hipMalloc, interleaved, ROUNDS rounds,
# headline encode only.  Usage (via gpurun): bash tools/ab_alloc.sh [ROUNDS] [bench args]
set -o pipefail
ROUNDS=${1:-3}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for r in $(seq 1 "$ROUNDS"); do
  for a in hipmalloc contiguous; do
    line=$(timeout -k 10 120 python3 bench.py --no-extras --steps 30 --alloc $a "$@" 2>/dev/null) || { echo "FAILED $a"; exit 1; }
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('round $r', '$a'.ljust(11), d['config']['k'], d['config']['m'], d['config']['shard_bytes'], d['roofline']['frac'], d['config']['hbm_alloc'])" "$line"
  done
done
