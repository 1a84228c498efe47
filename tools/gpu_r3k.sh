#!/bin/bash
# Line-owner kernel occupancy A/B: LDS pads of 0 / 1 / 2.5 / 5 KiB per wave.
set -o pipefail
tag=${1:-r3k}
out=gpurun_out
mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for lib in java-reed-solomon-distributed-file-system_amd/lib/librsamd.so build/ab/pad1k/librsamd.so build/ab/pad2k5/librsamd.so build/ab/pad5k/librsamd.so; do
    timeout -k 10 300 python tools/chunk_group_probe.py --strides 1000 --reps 2 --lib $lib >> $out/cg_pad_$tag.txt 2>&1 || { echo "probe failed"; tail $out/cg_pad_$tag.txt; exit 1; }
  done
done
grep '^{' $out/cg_pad_$tag.txt
