#!/bin/bash
# Round-2 GPU session: smoke -> gpu tests -> bench (N=1) -> self-launched
# 2-rank bench on one GPU -> rocprofv3 kernel trace -> counter list.
# Every GPU step has its own time limit; the chain stops at the first failure.
# Usage (via gpurun): bash tools/gpu_r2.sh [tag]
set -o pipefail
TAG=${1:-r2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
echo "== cpu share: nproc=$(nproc) cpu.max=$(cat /sys/fs/cgroup/cpu.max 2>/dev/null) $(date +%T)"

if [ -z "$SKIP_TESTS" ]; then
echo "== smoke $(date +%T)"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 || { tail -30 "$OUT/smoke_$TAG.log"; exit 1; }
tail -2 "$OUT/smoke_$TAG.log"

echo "== pytest -m gpu $(date +%T)"
timeout -k 10 700 python3 -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
    > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { tail -40 "$OUT/pytest_gpu_$TAG.log"; exit 1; }
tail -3 "$OUT/pytest_gpu_$TAG.log"
fi

echo "== bench $(date +%T)"
timeout -k 10 400 python3 bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || { tail -30 "$OUT/bench_$TAG.err"; exit 1; }
cat "$OUT/bench_$TAG.json"

echo "== bench --gpus 2 self-launched, 2 ranks on one GPU $(date +%T)"
timeout -k 10 400 python3 bench.py --gpus 2 --stripes 512 --steps 10 --warmup 2 --cfg3-stripes 256 \
    > "$OUT/bench2_$TAG.json" 2> "$OUT/bench2_$TAG.err" || { tail -30 "$OUT/bench2_$TAG.err"; exit 1; }
cat "$OUT/bench2_$TAG.json"

if [ -z "$SKIP_PROF" ]; then
echo "== rocprofv3 kernel trace $(date +%T)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
    python3 "$R/bench.py" --steps 10 --warmup 2 --no-extras > "$OUT/prof_$TAG.log" 2>&1 || { tail -30 "$OUT/prof_$TAG.log"; exit 1; }
find "$OUT/prof_$TAG" -name "*stats*"
timeout -k 10 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
fi
echo "== done $(date +%T)"
