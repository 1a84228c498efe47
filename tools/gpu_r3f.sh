#!/bin/bash
# Round 3: host-path bisect, line-owner kernel variants A/B (one process per
# build, alternated), PMC traffic of the line-owner encode.
set -o pipefail
tag=${1:-r3f}
out=gpurun_out
mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python tools/host_bisect.py > $out/host_bisect_$tag.txt 2>&1 || { echo "bisect failed"; tail $out/host_bisect_$tag.txt; exit 1; }
grep '^{' $out/host_bisect_$tag.txt
for rep in 1 2; do
  for lib in java-reed-solomon-distributed-file-system_amd/lib/librsamd.so build/ab/pw2/librsamd.so build/ab/norw/librsamd.so build/ab/plain/librsamd.so; do
    timeout -k 10 300 python tools/chunk_group_probe.py --strides 1000 --reps 2 --lib $lib >> $out/cg_variants_$tag.txt 2>&1 || { echo "probe failed"; tail $out/cg_variants_$tag.txt; exit 1; }
  done
done
grep '^{' $out/cg_variants_$tag.txt
export TMPDIR=/tmp
for W in cgenc cgdec01; do
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
cat $out/pmc_traffic_$tag.json
