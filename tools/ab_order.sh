#!/bin/bash
# A/B of the kernels' block order (kernels.hip block_item): GPU parity tests
# with the default order, then the bench line under each RSAMD_BLOCK_* setting.
# Usage (via gpurun): bash tools/ab_order.sh TAG
set -o pipefail
TAG=${1:-ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/order_$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for cfg in "ROT=0 XCD=0" "default" "ROT=3" "ROT=31" "ROT=0 XCD=0" "default"; do
  envs=""
  [ "$cfg" != default ] && for kv in $cfg; do envs="$envs RSAMD_BLOCK_$kv"; done
  name=$(echo "$cfg" | tr ' =' '_-')
  env $envs timeout -k 10 300 python3 bench.py --cpu-seconds 0.2 > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" \
      || { tail -20 "$OUT/bench_$name.err"; exit 1; }
  python3 - "$OUT/bench_$name.json" "$cfg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
e = d["extra"]
keys = ["decode_0_1_hbm_frac", "cfg3_10p4_4MiB_x128_encode_hbm_frac", "cfg3_10p4_4MiB_x128_decode_hbm_frac",
        "cfg3_10p4_4MiB_x128_pad4K_encode_hbm_frac", "cfg4_4p2_4KiB_x1M_encode_hbm_frac",
        "cfg4_4p2_4KiB_x1M_decode_hbm_frac", "cfg4_4p2_4KiB_x1M_decode_masked_bits_hbm_frac"]
print(f"{sys.argv[2]:12s} encode {d['roofline']['frac']:.4f} " + " ".join(f"{k.split('_hbm')[0][-22:]}={e[k]:.4f}" for k in keys))
PY
done
