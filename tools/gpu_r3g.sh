#!/bin/bash
# Line-owner kernel: aligned whole-line reads (variant ar) against the
# in-tree build, PMC traffic of both, and the TCC counter names of this GPU.
set -o pipefail
tag=${1:-r3g}
out=gpurun_out
mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 120 rocprofv3 --list-avail > $out/rocprof_list_avail.txt 2>&1 || echo "list-avail rc $?"
for rep in 1 2; do
  for lib in java-reed-solomon-distributed-file-system_amd/lib/librsamd.so build/ab/ar/librsamd.so; do
    timeout -k 10 300 python tools/chunk_group_probe.py --strides 1000 --reps 2 --lib $lib >> $out/cg_ar_$tag.txt 2>&1 || { echo "probe failed"; tail $out/cg_ar_$tag.txt; exit 1; }
  done
done
grep '^{' $out/cg_ar_$tag.txt
export TMPDIR=/tmp
for V in intree:java-reed-solomon-distributed-file-system_amd/lib/librsamd.so ar:build/ab/ar/librsamd.so; do
  n=${V%%:*}; lib=${V#*:}
  W=cgenc
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$out/pmcw_${tag}_${n}_$C" -o run -- \
        python3 tools/pmc_workloads.py $W $lib > "$out/pmcw_${tag}_${n}_$C.log" 2>&1 || { tail -20 "$out/pmcw_${tag}_${n}_$C.log"; exit 1; }
  done
  meta=$(grep '^{' "$out/pmcw_${tag}_${n}_FETCH_SIZE.log" | tail -1)
  kern=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['kernel'])" "$meta")
  alg=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['alg_bytes_per_launch'])" "$meta")
  python3 tools/pmc_summary.py "${W}_$n" "$kern" "$alg" "$out/pmcw_${tag}_${n}_FETCH_SIZE" "$out/pmcw_${tag}_${n}_WRITE_SIZE" \
      "$out/pmc_traffic_$tag.json" || exit 1
done
