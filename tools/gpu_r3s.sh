#!/bin/bash
set -o pipefail
out=gpurun_out; mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for pad in 0 4 16 64 128 1; do
    timeout -k 10 200 python tools/dec_probe.py --rounds 1 --row-pad $pad >> $out/dec_pad_$1.txt 2>&1 || { tail $out/dec_pad_$1.txt; exit 1; }
  done
done
grep '^{' $out/dec_pad_$1.txt
