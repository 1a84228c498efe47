#!/bin/bash
set -o pipefail
out=gpurun_out; mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
for n in 0 1 2 3 4 5; do
  for lib in build/ab/m0/librsamd.so java-reed-solomon-distributed-file-system_amd/lib/librsamd.so build/ab/m2/librsamd.so build/ab/m3/librsamd.so; do
    timeout -k 10 120 python tools/host_queues.py $n $lib >> $out/host_queues_$1.txt 2>&1 || { tail $out/host_queues_$1.txt; exit 1; }
  done
done
grep '^{' $out/host_queues_$1.txt
