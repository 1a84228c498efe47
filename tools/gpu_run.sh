#!/bin/bash
# The one GPU-box runner (via gpurun): bash tools/gpu_run.sh TAG STEP [STEP ...]
# Steps, run in the order given, each under its own time limit; the chain stops
# at the first failure (nothing more touches the GPU after a fault or timeout):
#   tests      pytest -m gpu (one process)              -> pytest_gpu_TAG.log
#   bounds     pytest -m gpu against the bounds-checking build (lib/bounds), serialised
#   hosttests  the host-buffer test files only           -> pytest_host_TAG.log
#   smoke      __graft_entry__.smoke()                  -> smoke_TAG.log
#   bench      bench.py at N = 1 (live PMC passes)      -> bench_TAG.json
#   prof       rocprofv3 --kernel-trace --stats of the headline -> prof_TAG/
#   rehearse   bench.py --gpus 2 and --gpus 4 with every leg, wall times -> bench{2,4}_TAG.json
#   pmc        FETCH/WRITE_SIZE passes of the chunk-group kernels -> pmc_traffic_TAG.json
#   probe:ARGS python3 ARGS (a tools/ probe)            -> probe_TAG_N.txt
#   kprobe:ARGS the same under rocprofv3 --kernel-trace --stats -> kprobe_TAG_N/, kprobe_TAG_N.txt
#   pmcc:W:C1,C2,...  one rocprofv3 --pmc pass of the given counters over pmc_workloads.py W -> pmcc_TAG.txt
set -o pipefail
tag=${1:?tag}
shift
out=gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $out
export TMPDIR=/tmp
# heartbeat: long legs print nothing for minutes
(while true; do date +%T > $out/.heartbeat_$tag; sleep 30; done) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
np=0
for step in "$@"; do
  echo "== $step $(date +%T)"
  t0=$(date +%s)
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
          > $out/pytest_gpu_$tag.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest_gpu_$tag.log; exit 1; }
      tail -1 $out/pytest_gpu_$tag.log ;;
    bounds)
      # kernels and copies serialised: a fault surfaces at the call that made it
      AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3 \
      RSAMD_TEST_LIB=java-reed-solomon-distributed-file-system_amd/lib/bounds/librsamd.so \
        timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
          > $out/pytest_bounds_$tag.log 2>&1 || { echo "bounds pytest failed"; tail -40 $out/pytest_bounds_$tag.log; exit 1; }
      tail -1 $out/pytest_bounds_$tag.log ;;
    hosttests)
      # the host-buffer paths only (direct, mirrored, staged; file layout), product library
      timeout -k 10 600 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_host_pageable.py \
          tests/test_gpu_random.py tests/test_gpu_file_random.py tests/test_gpu_jni_core.py -m gpu -x -v \
          --timeout 300 --timeout-method thread > $out/pytest_host_$tag.log 2>&1 \
          || { echo "host pytest failed"; tail -40 $out/pytest_host_$tag.log; exit 1; }
      tail -1 $out/pytest_host_$tag.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke_$tag.log 2>&1 \
          || { echo "smoke failed"; cat $out/smoke_$tag.log; exit 1; }
      tail -1 $out/smoke_$tag.log ;;
    bench)
      timeout -k 10 900 python bench.py > $out/bench_$tag.json 2> $out/bench_$tag.err \
          || { echo "bench failed"; tail -30 $out/bench_$tag.err; exit 1; } ;;
    prof)
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_$tag" -o run -- \
          python3 bench.py --no-extras --no-live-pmc > $out/bench_prof_$tag.json 2> $out/bench_prof_$tag.err \
          || { echo "prof failed"; tail -30 $out/bench_prof_$tag.err; exit 1; } ;;
    rehearse)
      for n in 2 4; do
        s0=$(date +%s)
        timeout -k 10 1000 python bench.py --gpus $n > $out/bench${n}_$tag.json 2> $out/bench${n}_$tag.err \
            || { echo "bench$n failed"; tail -30 $out/bench${n}_$tag.err; exit 1; }
        echo "bench --gpus $n wall $(( $(date +%s) - s0 )) s" | tee -a $out/rehearse_wall_$tag.txt
      done ;;
    pmc)
      for W in cgenc cgdec01 cgmaskbits; do
        for C in FETCH_SIZE WRITE_SIZE; do
          timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$out/pmcw_${tag}_${W}_$C" -o run -- \
              python3 tools/pmc_workloads.py $W > "$out/pmcw_${tag}_${W}_$C.log" 2>&1 || { tail -20 "$out/pmcw_${tag}_${W}_$C.log"; exit 1; }
        done
        meta=$(grep '^{' "$out/pmcw_${tag}_${W}_FETCH_SIZE.log" | tail -1)
        kern=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['kernel'])" "$meta")
        alg=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['alg_bytes_per_launch'])" "$meta")
        python3 tools/pmc_summary.py "$W" "$kern" "$alg" "$out/pmcw_${tag}_${W}_FETCH_SIZE" \
            "$out/pmcw_${tag}_${W}_WRITE_SIZE" "$out/pmc_traffic_$tag.json" || exit 1
      done ;;
    pmcw:*)  # pmcw:WORKLOAD[:LIB] -> FETCH/WRITE passes of one tools/pmc_workloads.py workload
      spec=${step#pmcw:}; W=${spec%%:*}; L=""; [ "$spec" != "$W" ] && L=${spec#*:}
      sfx=$W; [ -n "$L" ] && sfx=${W}_$(basename $(dirname $L))
      for C in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$out/pmcw_${tag}_${sfx}_$C" -o run -- \
            python3 tools/pmc_workloads.py $W $L > "$out/pmcw_${tag}_${sfx}_$C.log" 2>&1 || { tail -20 "$out/pmcw_${tag}_${sfx}_$C.log"; exit 1; }
      done
      meta=$(grep '^{' "$out/pmcw_${tag}_${sfx}_FETCH_SIZE.log" | tail -1)
      kern=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['kernel'])" "$meta")
      alg=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['alg_bytes_per_launch'])" "$meta")
      python3 tools/pmc_summary.py "$sfx" "$kern" "$alg" "$out/pmcw_${tag}_${sfx}_FETCH_SIZE" \
          "$out/pmcw_${tag}_${sfx}_WRITE_SIZE" "$out/pmc_traffic_$tag.json" || exit 1 ;;
    pmcc:*)  # pmcc:WORKLOAD:C1,C2,... -> one rocprofv3 --pmc pass of tools/pmc_workloads.py WORKLOAD
      np=$((np + 1))
      spec=${step#pmcc:}; W=${spec%%:*}; CS=${spec#*:}
      timeout -s KILL 120 rocprofv3 --pmc ${CS//,/ } --output-format csv -d "$out/pmcc_${tag}_$np" -o run -- \
          python3 tools/pmc_workloads.py $W > "$out/pmcc_${tag}_$np.log" 2>&1 || { tail -20 "$out/pmcc_${tag}_$np.log"; exit 1; }
      meta=$(grep '^{' "$out/pmcc_${tag}_$np.log" | tail -1)
      kern=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['kernel'])" "$meta")
      echo "$meta $(python3 tools/pmc_counters.py "$out/pmcc_${tag}_$np" "$kern")" | tee -a $out/pmcc_$tag.txt ;;
    probe:*)
      np=$((np + 1))
      timeout -k 10 600 python3 ${step#probe:} > $out/probe_${tag}_$np.txt 2>&1 \
          || { echo "probe failed"; tail -30 $out/probe_${tag}_$np.txt; exit 1; }
      tail -5 $out/probe_${tag}_$np.txt ;;
    kprobe:*)  # a tools/ probe under rocprofv3 --kernel-trace --stats -> kprobe_TAG_N/ + .txt
      np=$((np + 1))
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kprobe_${tag}_$np" -o run -- \
          python3 ${step#kprobe:} > $out/kprobe_${tag}_$np.txt 2>&1 \
          || { echo "kprobe failed"; tail -30 $out/kprobe_${tag}_$np.txt; exit 1; }
      grep '^{' $out/kprobe_${tag}_$np.txt | tail -12 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "   $step: $(( $(date +%s) - t0 )) s"
done
echo "== done $(date +%T)"
