#!/bin/bash
# Placement probe with VA logging, then the same under UTCL1 (TLB) counters plus a
# kernel trace (counter collection + kernel trace only).  Usage: bash tools/gpu_tlb.sh <tag>
set -o pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
export TMPDIR=/tmp
SP=0,0.5,1,2,3,5,8,13,21,34
AL=contiguous,contiguous,contiguous,contiguous,contiguous,contiguous,contiguous,contiguous,contiguous,contiguous
echo "== 4+2 placements with VA $(date +%T)"
ALLOCS=$AL SPACERS=$SP ORDERS=table timeout -k 10 200 python3 tools/placement_probe.py > "$OUT/placement_va_c2_$TAG.txt" 2>&1 || { tail -20 "$OUT/placement_va_c2_$TAG.txt"; exit 1; }
cat "$OUT/placement_va_c2_$TAG.txt"
echo "== 10+4 x1024 placements with VA $(date +%T)"
K=10 M=4 SHARD=$((4 << 20)) STRIPES=1024 ALLOCS=$AL SPACERS=$SP ORDERS=xcd timeout -k 10 200 python3 tools/placement_probe.py > "$OUT/placement_va_cfg3_$TAG.txt" 2>&1 || { tail -20 "$OUT/placement_va_cfg3_$TAG.txt"; exit 1; }
cat "$OUT/placement_va_cfg3_$TAG.txt"
echo "== 4+2 placements under UTCL1 counters $(date +%T)"
ALLOCS=$AL SPACERS=$SP ORDERS=table timeout -s KILL 240 rocprofv3 --kernel-trace \
  --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum \
  --output-format csv -d "$OUT/tlb_$TAG" -o run -- python3 "$R/tools/placement_probe.py" > "$OUT/tlb_$TAG.log" 2>&1 || { tail -20 "$OUT/tlb_$TAG.log"; exit 1; }
grep '^{' "$OUT/tlb_$TAG.log"
echo "== done $(date +%T)"
