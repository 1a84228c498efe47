#!/bin/bash
# Unified line-owner kernel (uniform plans with any output set, and per-group
# records): full GPU tests, then the chunk-group probe, in-tree vs the 8-byte
# kernels (TUNING build, RSAMD_GROUP8=0).
set -o pipefail
tag=${1:-r3i}
out=gpurun_out
mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu_$tag.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest_gpu_$tag.log; exit 1; }
tail -2 $out/pytest_gpu_$tag.log
for rep in 1 2; do
  timeout -k 10 300 python tools/chunk_group_probe.py --strides 1000 --reps 2 >> $out/cg_$tag.txt 2>&1 || { echo "probe failed"; tail $out/cg_$tag.txt; exit 1; }
  RSAMD_GROUP8=0 timeout -k 10 300 python tools/chunk_group_probe.py --strides 1000 --reps 2 --lib build/ab/tuning/librsamd.so >> $out/cg_$tag.txt 2>&1 || { echo "probe2 failed"; tail $out/cg_$tag.txt; exit 1; }
done
grep '^{' $out/cg_$tag.txt
