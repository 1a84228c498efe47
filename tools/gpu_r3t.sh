#!/bin/bash
set -o pipefail
out=gpurun_out; mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
RSAMD_TEST_LIB=build/ab/early/librsamd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_recovery.py tests/test_gpu_granule.py -x -q --timeout 120 --timeout-method thread > $out/pytest_early_$1.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_early_$1.log; exit 1; }
tail -1 $out/pytest_early_$1.log
timeout -k 10 600 python tools/masked_ab.py java-reed-solomon-distributed-file-system_amd/lib/librsamd.so build/ab/early/librsamd.so --reps 3 > $out/masked_early_$1.txt 2>&1 || { tail $out/masked_early_$1.txt; exit 1; }
cat $out/masked_early_$1.txt
