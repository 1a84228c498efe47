#!/bin/bash
# Round 3: line-owner chunk-group kernel parity + A/B against the 8-byte
# kernels (RSAMD_GROUP8=0 in a TUNING build), then a trace of the host path.
set -o pipefail
tag=${1:-r3c}
out=gpurun_out
mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_chunk_groups.py tests/test_gpu_recovery.py -x -q --timeout 120 --timeout-method thread > $out/pytest_cg_$tag.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest_cg_$tag.log; exit 1; }
tail -2 $out/pytest_cg_$tag.log
for rep in 1 2; do
  timeout -k 10 300 python tools/chunk_group_probe.py --strides 1000 --reps 3 >> $out/cg_group8_$tag.txt 2>&1 || { echo "probe failed"; tail $out/cg_group8_$tag.txt; exit 1; }
  RSAMD_GROUP8=0 timeout -k 10 300 python tools/chunk_group_probe.py --strides 1000 --reps 3 --lib build/ab/tuning/librsamd.so >> $out/cg_group8_$tag.txt 2>&1 || { echo "probe2 failed"; tail $out/cg_group8_$tag.txt; exit 1; }
done
cat $out/cg_group8_$tag.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/host_trace_$tag" -o run -- python "$GRAFT_REPO_ROOT/tools/host_trace.py" > "$GRAFT_REPO_ROOT/$out/host_trace_$tag.txt" 2>&1 || { echo "trace failed"; tail "$GRAFT_REPO_ROOT/$out/host_trace_$tag.txt"; exit 1; }
grep '^{' "$GRAFT_REPO_ROOT/$out/host_trace_$tag.txt"
cd "$GRAFT_REPO_ROOT" && timeout -k 10 120 python tools/host_trace.py --calls 6 > $out/host_untraced_$tag.txt 2>&1 && cat $out/host_untraced_$tag.txt
