#!/bin/bash
# One GPU-box session: smoke -> gpu tests -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; the chain stops at the first failure.
# Usage (from the repo root, via gpurun):  bash tools/gpu_round.sh [tag]
set -o pipefail
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"

echo "== smoke $(date +%T)"
timeout -k 10 400 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 || { tail -30 "$OUT/smoke_$TAG.log"; exit 1; }
tail -2 "$OUT/smoke_$TAG.log"

echo "== pytest -m gpu $(date +%T)"
timeout -k 10 700 python3 -u -m pytest tests -x -v -m gpu --timeout 150 --timeout-method thread \
    > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { tail -40 "$OUT/pytest_gpu_$TAG.log"; exit 1; }
tail -3 "$OUT/pytest_gpu_$TAG.log"

echo "== bench $(date +%T)"
timeout -k 10 400 python3 bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || { tail -30 "$OUT/bench_$TAG.err"; exit 1; }
cat "$OUT/bench_$TAG.json"

echo "== 2-rank bench on one GPU (gloo; exercises the multi-rank path) $(date +%T)"
RSAMD_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --stripes 512 --steps 5 --warmup 2 --no-extras \
    > "$OUT/bench2rank_$TAG.json" 2> "$OUT/bench2rank_$TAG.err" || { tail -30 "$OUT/bench2rank_$TAG.err"; exit 1; }
cat "$OUT/bench2rank_$TAG.json"

echo "== rocprofv3 kernel trace $(date +%T)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
    python3 "$R/bench.py" --steps 10 --warmup 2 --no-extras > "$OUT/prof_$TAG.log" 2>&1 || { tail -30 "$OUT/prof_$TAG.log"; exit 1; }
find "$OUT/prof_$TAG" -name "*stats*" | head
echo "== done $(date +%T)"
