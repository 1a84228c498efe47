#!/bin/bash
# PMC passes for the bench workload: FETCH_SIZE and WRITE_SIZE in separate runs
# (counter collection only: no sys/runtime trace), for the headline batch in
# the granule layout (bench.py's default) and in the packed layout, then the
# summaries into profiles/pmc_traffic.json.  Usage (via gpurun): bash tools/gpu_pmc.sh [tag]
set -o pipefail
TAG=${1:-r1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
ALG=$((6*1048576*4096))
for LAYOUT in granule packed; do
  ARGS="--steps 3 --warmup 1 --no-extras --layout $LAYOUT"
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "== pmc $LAYOUT $C $(date +%T)"
    timeout -k 10 400 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${TAG}_${LAYOUT}_$C" -o run -- \
        python3 "$R/bench.py" $ARGS > "$OUT/pmc_${TAG}_${LAYOUT}_$C.log" 2>&1 || { tail -30 "$OUT/pmc_${TAG}_${LAYOUT}_$C.log"; exit 1; }
  done
  SUF=""
  [ "$LAYOUT" = granule ] && SUF="_granule65536"
  python3 tools/pmc_summary.py encode_4_2_1048576_4096$SUF "gf_vec_kernel<4, 2, false>" $ALG \
      "$OUT/pmc_${TAG}_${LAYOUT}_FETCH_SIZE" "$OUT/pmc_${TAG}_${LAYOUT}_WRITE_SIZE" "$OUT/pmc_traffic.json"
  python3 tools/pmc_summary.py verify_4_2_1048576_4096$SUF "gf_vec_kernel<4, 2, true>" $ALG \
      "$OUT/pmc_${TAG}_${LAYOUT}_FETCH_SIZE" "$OUT/pmc_${TAG}_${LAYOUT}_WRITE_SIZE" "$OUT/pmc_traffic.json"
done
echo "== done $(date +%T)"
