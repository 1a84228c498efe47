#!/bin/bash
# PMC traffic of every measured kernel shape besides the headline encode
# (tools/gpu_pmc.sh): one process per workload (tools/pmc_workloads.py) under
# FETCH_SIZE and under WRITE_SIZE (separate runs, counters only), summarised
# into gpurun_out/pmc_traffic_all.json.  Usage (via gpurun): bash tools/gpu_pmc_all.sh [tag]
set -o pipefail
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
for W in ${WORKLOADS:-dec42_01 enc104 dec104 enc42_4k maskbits fenc fdec_05}; do
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "== $W $C $(date +%T)"
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmcw_${TAG}_${W}_$C" -o run -- \
        python3 "$R/tools/pmc_workloads.py" $W > "$OUT/pmcw_${TAG}_${W}_$C.log" 2>&1 || { tail -20 "$OUT/pmcw_${TAG}_${W}_$C.log"; exit 1; }
  done
  meta=$(grep '^{' "$OUT/pmcw_${TAG}_${W}_FETCH_SIZE.log" | tail -1)
  kern=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['kernel'])" "$meta")
  alg=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['alg_bytes_per_launch'])" "$meta")
  python3 tools/pmc_summary.py "$W" "$kern" "$alg" "$OUT/pmcw_${TAG}_${W}_FETCH_SIZE" "$OUT/pmcw_${TAG}_${W}_WRITE_SIZE" \
      "$OUT/pmc_traffic_all.json" || exit 1
done
echo "== done $(date +%T)"
