#!/bin/bash
# XOR-network vs table kernels: kernel trace (durations, VGPR/SGPR) and SQ
# counters of both, on the headline and config[3] shapes.
set -o pipefail
TAG=${1:-r2c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
for X in 1 0; do
  for W in enc42 enc104; do
    echo "== trace $W xornet=$X $(date +%T)"
    RSAMD_XORNET=$X timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_${TAG}_${W}_x$X" -o run -- \
        python3 "$R/tools/pmc_workloads.py" $W > "$OUT/kt_${TAG}_${W}_x$X.log" 2>&1 || { tail -20 "$OUT/kt_${TAG}_${W}_x$X.log"; exit 1; }
  done
  RSAMD_XORNET=$X WORKLOADS="enc42 enc104" bash tools/gpu_sq.sh $TAG || exit 1
done
python3 - "$OUT" "$TAG" <<'PY'
import csv, glob, sys
out, tag = sys.argv[1], sys.argv[2]
for p in sorted(glob.glob(f"{out}/kt_{tag}_*/**/*kernel_trace.csv", recursive=True)):
    rows = [r for r in csv.DictReader(open(p)) if "xornet" in r["Kernel_Name"] or "gf_vec_kernel" in r["Kernel_Name"]]
    for r in rows[-2:]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        print(p.split("/")[-3], r["Kernel_Name"][:60], "ms=%.3f" % d, "vgpr", r.get("VGPR_Count"), "agpr", r.get("Accum_VGPR_Count"), "sgpr", r.get("SGPR_Count"), "scratch", r.get("Scratch_Size"), "lds", r.get("LDS_Block_Size", r.get("Lds_Size")))
PY
echo "== done $(date +%T)"
