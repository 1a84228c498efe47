#!/bin/bash
# Round-3 GPU pass: GPU tests, smoke, the bench at N = 1, and a 2-rank
# rehearsal on the one GPU (gloo).  Each step has its own limit; the first
# failure ends the run.  Usage: tools/gpu_r3.sh TAG
set -o pipefail
tag=${1:-r3}
out=gpurun_out
mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu_$tag.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_gpu_$tag.log; exit 1; }
tail -3 $out/pytest_gpu_$tag.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke_$tag.log 2>&1 || { echo "smoke failed"; cat $out/smoke_$tag.log; exit 1; }
timeout -k 10 900 python bench.py > $out/bench_$tag.json 2> $out/bench_$tag.err || { echo "bench failed"; tail -30 $out/bench_$tag.err; exit 1; }
echo bench done
timeout -k 10 900 python bench.py --gpus 2 > $out/bench2_$tag.json 2> $out/bench2_$tag.err || { echo "bench2 failed"; tail -30 $out/bench2_$tag.err; exit 1; }
echo bench2 done
