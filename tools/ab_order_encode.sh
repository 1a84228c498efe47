#!/bin/bash
# Interleaved A/B of the block order on the headline encode (bench.py
# --no-extras, 30 timed steps), ROUNDS rounds over the configurations.
# Usage (via gpurun): [CONFIGS="ROT=0,XCD=0 ROT=127,XCD=0 ..."] bash tools/ab_order_encode.sh [ROUNDS] [extra bench args]
set -o pipefail
ROUNDS=${1:-3}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for r in $(seq 1 "$ROUNDS"); do
  CONFIGS=${CONFIGS:-ROT=0,XCD=0 ROT=31,XCD=0 ROT=0,XCD=1 ROT=31,XCD=1 ROT=7,XCD=0 ROT=127,XCD=0}
  for cfg in $CONFIGS; do
    cfg=${cfg//,/ }
    envs=""
    for kv in $cfg; do envs="$envs RSAMD_BLOCK_$kv"; done
    line=$(env $envs timeout -k 10 120 python3 bench.py --no-extras --steps 30 "$@" 2>/dev/null) || { echo "FAILED: $cfg"; exit 1; }
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('round $r', '$cfg'.ljust(14), d['config']['k'], d['config']['m'], d['config']['shard_bytes'], d['roofline']['frac'])" "$line"
  done
done
