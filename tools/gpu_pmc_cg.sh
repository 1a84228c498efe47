# PMC traffic (FETCH_SIZE, WRITE_SIZE passes) of chunk-group workloads (tools/pmc_workloads.py).
# Usage (via gpurun): bash tools/gpu_pmc_cg.sh TAG [WORKLOAD ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out; tag=${1:-r3zd}
shift || true
for W in ${@:-cgdec05 cgdec15 cgdec01}; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$out/pmcw_${tag}_${W}_$C" -o run -- \
        python3 tools/pmc_workloads.py $W > "$out/pmcw_${tag}_${W}_$C.log" 2>&1 || { tail -20 "$out/pmcw_${tag}_${W}_$C.log"; exit 1; }
  done
  meta=$(grep '^{' "$out/pmcw_${tag}_${W}_FETCH_SIZE.log" | tail -1)
  kern=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['kernel'])" "$meta")
  alg=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['alg_bytes_per_launch'])" "$meta")
  python3 tools/pmc_summary.py "$W" "$kern" "$alg" "$out/pmcw_${tag}_${W}_FETCH_SIZE" "$out/pmcw_${tag}_${W}_WRITE_SIZE" \
      "$out/pmc_traffic_$tag.json" || exit 1
done
