#!/bin/bash
# A/B of the fused file kernels (tiled vs untiled encode and decode, block 1000 vs
# 1024): timing JSON plus per-kernel FETCH_SIZE / WRITE_SIZE (separate --pmc
# passes) under gpurun_out/ab/.
set -e
mkdir -p gpurun_out/ab
export TMPDIR=/tmp RSAMD_BENCH_SKIP_MASKED=1
for B in ${AB_BLOCKS:-1000 1024}; do for M in ${AB_MODES:-1 0}; do
  tag=b${B}_m${M}
  RSAMD_BENCH_BLOCK=$B RSAMD_FILE_DECODE=$M RSAMD_FILE_ENCODE=$M timeout -k 10 240 python3 tools/layout_bench.py > gpurun_out/ab/$tag.json
  [ -n "$AB_NO_PMC" ] && continue
  for C in FETCH_SIZE WRITE_SIZE; do
    RSAMD_BENCH_BLOCK=$B RSAMD_FILE_DECODE=$M RSAMD_FILE_ENCODE=$M timeout -k 10 300 rocprofv3 --pmc $C --output-format csv \
      -d gpurun_out/ab/${tag}_$C -o run -- python3 tools/layout_bench.py > gpurun_out/ab/${tag}_$C.log 2>&1
  done
done; done
for f in gpurun_out/ab/*.json; do echo "$f $(cat $f)"; done
[ -n "$AB_NO_PMC" ] || python3 tools/pmc_kernels.py gpurun_out/ab/*_SIZE
