#!/bin/bash
set -o pipefail
out=gpurun_out; mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
for c in 4 6 8 10; do
  RSAMD_CHUNKS=$c timeout -k 10 120 python tools/host_queues.py 0 build/ab/tuning/librsamd.so | sed "s/^{/{\"chunks\": $c, /" >> $out/host_chunks_$1.txt 2>&1 || { tail $out/host_chunks_$1.txt; exit 1; }
done
done
grep '^{' $out/host_chunks_$1.txt
timeout -k 10 120 python tools/host_trace.py --calls 6 > $out/host_untraced_$1.txt 2>&1 && cat $out/host_untraced_$1.txt
