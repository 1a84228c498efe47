#!/bin/bash
# A/B of the tiled file decode's workgroup shape (layout.hip
# file_decode_tiled_kernel<K, E, THREADS, SLOTS>, RSAMD_DEC_TILE=threads,slots):
# GPU layout tests under each non-default shape, then tools/layout_bench.py's
# file legs per shape, twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
SHAPES=${SHAPES:-"256,2 256,1 512,1 128,2 512,2"}
for t in $SHAPES; do
  RSAMD_DEC_TILE=$t timeout -k 10 300 python3 -u -m pytest tests/test_gpu_layout.py -x -q -m gpu --timeout 150 \
      --timeout-method thread 2>&1 | tail -1 | sed "s/^/tests $t: /" || exit 1
done
for r in 1 2; do
  for t in $SHAPES; do
    line=$(RSAMD_DEC_TILE=$t RSAMD_BENCH_SKIP_MASKED=1 timeout -k 10 200 python3 tools/layout_bench.py 2>/dev/null) || { echo "FAILED $t"; exit 1; }
    echo "round $r tile $t $line"
  done
done
