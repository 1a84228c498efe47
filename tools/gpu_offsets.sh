#!/bin/bash
# Rate vs base offset inside one contiguous range (tools/offset_probe.py).
# Usage (via gpurun): bash tools/gpu_offsets.sh <tag>
set -o pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
echo "== 4+2 x 1 MiB x 4096, 256 MiB steps over 16 GiB $(date +%T)"
timeout -k 10 200 python3 tools/offset_probe.py > "$OUT/offsets_c2_$TAG.txt" 2>&1 || { tail -20 "$OUT/offsets_c2_$TAG.txt"; exit 1; }
echo "== 4+2, 2 MiB steps over 64 MiB $(date +%T)"
SLACK_GIB=0.0625 STEP_MIB=2 timeout -k 10 200 python3 tools/offset_probe.py > "$OUT/offsets_c2_fine_$TAG.txt" 2>&1 || { tail -20 "$OUT/offsets_c2_fine_$TAG.txt"; exit 1; }
echo "== 10+4 x 4 MiB x 1024, 256 MiB steps over 16 GiB $(date +%T)"
K=10 M=4 SHARD=$((4 << 20)) STRIPES=1024 timeout -k 10 300 python3 tools/offset_probe.py > "$OUT/offsets_cfg3_$TAG.txt" 2>&1 || { tail -20 "$OUT/offsets_cfg3_$TAG.txt"; exit 1; }
echo "== done $(date +%T)"
