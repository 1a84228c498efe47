#!/bin/bash
# Block order vs pool placement (tools/placement_probe.py): config[3] 10+4 x 4 MiB x 1024
# and the 4+2 x 1 MiB x 4096 headline, each on contiguous pools placed after spacers.
# Usage (via gpurun): bash tools/gpu_placement.sh <tag>
set -o pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
SP=0,0.5,1,2,3,5,8,13
AL=contiguous,contiguous,contiguous,contiguous,contiguous,contiguous,contiguous,contiguous
echo "== 10+4 x 4 MiB x 1024 $(date +%T)"
K=10 M=4 SHARD=$((4 << 20)) STRIPES=1024 ALLOCS=$AL SPACERS=$SP ORDERS=xcd,rot1535,xcd_rot1535,stripe_major \
  timeout -k 10 300 python3 tools/placement_probe.py > "$OUT/placement_cfg3_$TAG.txt" 2>&1 || { tail -20 "$OUT/placement_cfg3_$TAG.txt"; exit 1; }
cat "$OUT/placement_cfg3_$TAG.txt"
echo "== 4+2 x 1 MiB x 4096 $(date +%T)"
ALLOCS=$AL SPACERS=$SP ORDERS=table,xcd,xcd_rot383,rot127 \
  timeout -k 10 300 python3 tools/placement_probe.py > "$OUT/placement_c2_$TAG.txt" 2>&1 || { tail -20 "$OUT/placement_c2_$TAG.txt"; exit 1; }
cat "$OUT/placement_c2_$TAG.txt"
echo "== done $(date +%T)"
