#!/bin/bash
# Closing evidence for a round: smoke, every GPU test, the bench (N=1 and the
# self-launched 2-rank run on one GPU), the rocprofv3 kernel trace of the
# headline, and its PMC HBM traffic (tools/gpu_pmc.sh).  Each GPU step has its
# own time limit; the chain stops at the first failure.
# Usage (via gpurun): bash tools/gpu_r2_close.sh <tag>
set -o pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
SKIP_PROF=1 bash tools/gpu_r2.sh "$TAG" || exit 1
OUT=$R/gpurun_out
export TMPDIR=/tmp
echo "== rocprofv3 kernel trace $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
    python3 "$R/bench.py" --steps 20 --warmup 3 --no-extras > "$OUT/prof_$TAG.log" 2>&1 || { tail -30 "$OUT/prof_$TAG.log"; exit 1; }
grep '^{' "$OUT/prof_$TAG.log" | tail -1
bash tools/gpu_pmc.sh "$TAG" || exit 1
echo "== close done $(date +%T)"
