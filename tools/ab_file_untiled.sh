#!/bin/bash
# Untiled file decode A/B: GPU layout tests forced onto the untiled kernel, the
# full GPU suite, then tools/file_decode_untiled_probe.py on an older build
# (tools/bin/old/librsamd.so) and on the current one, twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
RSAMD_FILE_DECODE=0 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_layout.py -x -q -m gpu --timeout 120 --timeout-method thread \
    > "$OUT/pytest_layout_untiled.log" 2>&1 || { tail -30 "$OUT/pytest_layout_untiled.log"; exit 1; }
tail -1 "$OUT/pytest_layout_untiled.log"
timeout -k 10 300 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu_r1v.log" 2>&1 || { tail -30 "$OUT/pytest_gpu_r1v.log"; exit 1; }
tail -1 "$OUT/pytest_gpu_r1v.log"
for rep in 1 2; do
  echo old; RSAMD_FILE_DECODE=0 RSAMD_LIB_OVERRIDE=$R/tools/bin/old/librsamd.so timeout -k 10 120 python3 tools/file_decode_untiled_probe.py 2>/dev/null || exit 1
  echo new; RSAMD_FILE_DECODE=0 timeout -k 10 120 python3 tools/file_decode_untiled_probe.py 2>/dev/null || exit 1
done | tee "$OUT/file_untiled_ab.txt"
