#!/bin/bash
# A/B of librsamd.so builds (tools/bin/var_<name>/librsamd.so, built with
# `make OUT=... OBJ=... KDEFS=...` in csrc/) on the 10+4 legs: each variant is
# copied over the package library in this scratch copy of the tree, then
# tools/masked_ref_probe.py reports product/XOR-reference ratios on one pool.
# Usage (via gpurun): bash tools/gpu_variants.sh <tag> <variant> ...   ("base" = the tree's build)
set -o pipefail
TAG=${1:?tag}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
LIB=java-reed-solomon-distributed-file-system_amd/lib/librsamd.so
cp "$LIB" /tmp/librsamd_base.so
for V in "$@"; do
  if [ "$V" = base ]; then cp /tmp/librsamd_base.so "$LIB"; else cp "tools/bin/var_$V/librsamd.so" "$LIB"; fi
  echo "== $V $(date +%T)"
  timeout -k 10 200 python3 tools/masked_ref_probe.py 128 4 > "$OUT/var_${TAG}_$V.txt" 2>&1 || { tail -20 "$OUT/var_${TAG}_$V.txt"; cp /tmp/librsamd_base.so "$LIB"; exit 1; }
  python3 - "$OUT/var_${TAG}_$V.txt" <<'PY'
import json, sys, statistics
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
med = lambda k: statistics.median(r[k] for r in rows)
print(f"uniform {med('uniform'):.4f} (/ref {statistics.median(r['uniform']/r['uniform_ref'] for r in rows):.3f})  "
      f"masked {med('masked'):.4f} (/ref {statistics.median(r['masked']/r['masked_ref'] for r in rows):.3f})")
PY
done
cp /tmp/librsamd_base.so "$LIB"
echo "== done $(date +%T)"
