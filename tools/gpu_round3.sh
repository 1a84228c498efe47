#!/bin/bash
# Round-3 closing pass: GPU tests, smoke, the bench at N = 1 (with its live
# PMC passes), a rocprofv3 kernel-stats profile of the headline, the 2- and
# 4-rank rehearsals on the one GPU, PMC traffic of the chunk-group kernels.
# Usage (via gpurun): bash tools/gpu_round3.sh TAG
set -o pipefail
tag=${1:-r3}
out=gpurun_out
mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu_$tag.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest_gpu_$tag.log; exit 1; }
tail -1 $out/pytest_gpu_$tag.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke_$tag.log 2>&1 || { echo "smoke failed"; cat $out/smoke_$tag.log; exit 1; }
tail -1 $out/smoke_$tag.log
timeout -k 10 900 python bench.py > $out/bench_$tag.json 2> $out/bench_$tag.err || { echo "bench failed"; tail -30 $out/bench_$tag.err; exit 1; }
echo bench done
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_$tag" -o run -- python3 bench.py --no-extras --no-live-pmc > $out/bench_prof_$tag.json 2> $out/bench_prof_$tag.err || { echo "prof failed"; tail -30 $out/bench_prof_$tag.err; exit 1; }
echo prof done
timeout -k 10 900 python bench.py --gpus 2 > $out/bench2_$tag.json 2> $out/bench2_$tag.err || { echo "bench2 failed"; tail -30 $out/bench2_$tag.err; exit 1; }
echo bench2 done
timeout -k 10 900 python bench.py --gpus 4 --no-extras > $out/bench4_$tag.json 2> $out/bench4_$tag.err || { echo "bench4 failed"; tail -30 $out/bench4_$tag.err; exit 1; }
echo bench4 done
for W in cgenc cgdec01 cgmaskbits; do
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
