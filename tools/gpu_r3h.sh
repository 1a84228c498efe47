#!/bin/bash
# Line-owner kernel with aligned reads: parity of the ar2 build (chunk-group
# and recovery tests against it), then ar / ar2 / in-tree A/B and PMC of ar2.
set -o pipefail
tag=${1:-r3h}
out=gpurun_out
mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
RSAMD_TEST_LIB=build/ab/ar2/librsamd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_chunk_groups.py tests/test_gpu_recovery.py -x -q --timeout 120 --timeout-method thread > $out/pytest_ar2_$tag.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest_ar2_$tag.log; exit 1; }
tail -2 $out/pytest_ar2_$tag.log
for rep in 1 2; do
  for lib in build/ab/ar/librsamd.so build/ab/ar2/librsamd.so; do
    timeout -k 10 300 python tools/chunk_group_probe.py --strides 1000 --reps 2 --lib $lib >> $out/cg_ar2_$tag.txt 2>&1 || { echo "probe failed"; tail $out/cg_ar2_$tag.txt; exit 1; }
  done
done
grep '^{' $out/cg_ar2_$tag.txt
export TMPDIR=/tmp
for V in ar2:build/ab/ar2/librsamd.so; do
  n=${V%%:*}; lib=${V#*:}
  for W in cgenc cgdec01; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$out/pmcw_${tag}_${n}_${W}_$C" -o run -- \
        python3 tools/pmc_workloads.py $W $lib > "$out/pmcw_${tag}_${n}_${W}_$C.log" 2>&1 || { tail -20 "$out/pmcw_${tag}_${n}_${W}_$C.log"; exit 1; }
  done
  meta=$(grep '^{' "$out/pmcw_${tag}_${n}_${W}_FETCH_SIZE.log" | tail -1)
  kern=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['kernel'])" "$meta")
  alg=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['alg_bytes_per_launch'])" "$meta")
  python3 tools/pmc_summary.py "${W}_$n" "$kern" "$alg" "$out/pmcw_${tag}_${n}_${W}_FETCH_SIZE" "$out/pmcw_${tag}_${n}_${W}_WRITE_SIZE" \
      "$out/pmc_traffic_$tag.json" || exit 1
  done
done
