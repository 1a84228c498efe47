#!/bin/bash
set -o pipefail
out=gpurun_out; mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
for n in 0 1 2 3 4 5 6 7; do
  timeout -k 10 120 python tools/host_queues.py $n >> $out/host_queues_r3n.txt 2>&1 || { tail $out/host_queues_r3n.txt; exit 1; }
done
grep '^{' $out/host_queues_r3n.txt
