#!/bin/bash
# Round-3 evidence pass: the bench at N = 1 (its own live PMC passes), a
# rocprofv3 kernel-stats profile of the same command, the 2- and 4-rank
# rehearsals on the one GPU, and PMC traffic of the chunk-group kernels.
set -o pipefail
tag=${1:-r3m}
out=gpurun_out
mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 python bench.py > $out/bench_$tag.json 2> $out/bench_$tag.err || { echo "bench failed"; tail -30 $out/bench_$tag.err; exit 1; }
echo bench done
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_$tag" -o run -- python3 bench.py --no-extras --no-live-pmc > $out/bench_prof_$tag.json 2> $out/bench_prof_$tag.err || { echo "prof failed"; tail -30 $out/bench_prof_$tag.err; exit 1; }
echo prof done
timeout -k 10 900 python bench.py --gpus 2 > $out/bench2_$tag.json 2> $out/bench2_$tag.err || { echo "bench2 failed"; tail -30 $out/bench2_$tag.err; exit 1; }
echo bench2 done
timeout -k 10 900 python bench.py --gpus 4 --no-extras > $out/bench4_$tag.json 2> $out/bench4_$tag.err || { echo "bench4 failed"; tail -30 $out/bench4_$tag.err; exit 1; }
echo bench4 done
for W in cgenc cgdec01 cgmaskbits cgmaskbits1k; do
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
echo pmc done
