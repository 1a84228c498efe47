#!/bin/bash
set -o pipefail
out=gpurun_out; mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for lib in java-reed-solomon-distributed-file-system_amd/lib/librsamd.so build/ab/lds1/librsamd.so build/ab/lds2/librsamd.so build/ab/ldsp1k/librsamd.so; do
    timeout -k 10 300 python tools/chunk_group_probe.py --strides 1000 --reps 2 --lib $lib >> $out/cg_lds_$1.txt 2>&1 || { echo "probe failed"; tail $out/cg_lds_$1.txt; exit 1; }
  done
done
grep '^{' $out/cg_lds_$1.txt
