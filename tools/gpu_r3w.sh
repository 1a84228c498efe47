#!/bin/bash
set -o pipefail
out=gpurun_out; mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for lib in java-reed-solomon-distributed-file-system_amd/lib/librsamd.so build/ab/rp/librsamd.so; do
    timeout -k 10 200 python tools/dec_probe.py --rounds 1 --lib $lib >> $out/dec_rp_$1.txt 2>&1 || { tail $out/dec_rp_$1.txt; exit 1; }
  done
done
grep '^{' $out/dec_rp_$1.txt
