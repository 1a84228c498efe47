#!/bin/bash
# A/B of the file kernels' XCD block order (layout.hip file_block): GPU layout
# tests, then bench.py's file legs with RSAMD_FILE_XCD=0 and the default, twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_layout.py tests/test_wire.py -x -q -m gpu --timeout 150 \
    --timeout-method thread 2>&1 | tail -1 || exit 1
for r in 1 2; do
  for x in 0 1; do
    line=$(RSAMD_FILE_XCD=$x timeout -k 10 300 python3 bench.py --cpu-seconds 0.2 2>/dev/null) || { echo FAILED; exit 1; }
    python3 -c "import json,sys; e=json.loads(sys.argv[1])['extra']; print('round $r XCD=$x', 'file_encode', e['file_encode_hbm_frac'], 'file_decode', e['file_decode_hbm_frac'], 'rt', e['file_round_trip_ok'])" "$line"
  done
done
