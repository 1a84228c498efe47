#!/bin/bash
# k = 10 per-stripe-pattern decode: parity of both kernel choices
# (RSAMD_MASKED_WIDE = 0 runtime-k kernel, 1 compile-time gf_masked_kernel<10, M>)
# and their rate (tools/masked_wide_probe.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
for mode in 1 0; do
  RSAMD_MASKED_WIDE=$mode timeout -k 10 300 python3 -u -m pytest tests/test_gpu_recovery.py -x -q --timeout 120 --timeout-method thread -m gpu \
     > "$OUT/masked_pytest_$mode.log" 2>&1 || { tail -30 "$OUT/masked_pytest_$mode.log"; exit 1; }
  tail -1 "$OUT/masked_pytest_$mode.log"
done
for rep in 1 2; do for mode in 0 1; do
  echo "mode $mode"; RSAMD_MASKED_WIDE=$mode timeout -k 10 120 python3 tools/masked_wide_probe.py || exit 1
done; done 2>&1 | tee "$OUT/masked_wide_ab.txt"
