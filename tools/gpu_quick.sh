#!/bin/bash
# Short GPU check after a kernel change: the GPU parity suite, the bench line,
# and (optional) a microbenchmark binary from tools/bin.  Each step has its own
# time limit; the chain stops at the first failure.
# Usage (via gpurun): bash tools/gpu_quick.sh TAG [tools/bin/<microbench> args...]
set -o pipefail
TAG=${1:-q}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
echo "== pytest -m gpu $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread \
    > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { tail -40 "$OUT/pytest_gpu_$TAG.log"; exit 1; }
tail -2 "$OUT/pytest_gpu_$TAG.log"
if [ $# -gt 0 ]; then
  echo "== $* $(date +%T)"
  timeout -k 10 240 "$@" > "$OUT/micro_$TAG.txt" 2>&1 || { tail -30 "$OUT/micro_$TAG.txt"; exit 1; }
  cat "$OUT/micro_$TAG.txt"
fi
echo "== bench $(date +%T)"
timeout -k 10 400 python3 bench.py --cpu-seconds 2 > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || { tail -30 "$OUT/bench_$TAG.err"; exit 1; }
cat "$OUT/bench_$TAG.json"
echo "== done $(date +%T)"
