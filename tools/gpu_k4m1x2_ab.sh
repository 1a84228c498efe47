#!/bin/bash
# (gf_vec_k4m1x2_kernel and RSAMD_K4M1X2 were removed after this A/B, run r2bx: the
# two-chunk kernel lost; this script records how profiles/r2/ab/k4m1x2_ab_r2bx.txt was measured.)
# A/B of the two-chunk-per-wave kernel for one-output 4-input plans
# (gf_vec_k4m1x2_kernel; RSAMD_K4M1X2=0 keeps gf_vec_kernel<4,1>): GPU tests,
# then tools/granule_decode_probe.py (granule view, G = 64 KiB) and
# tools/lib_ab_same.py (packed shapes) with the knob off and on, alternated.
# Usage (via gpurun): bash tools/gpu_k4m1x2_ab.sh TAG
set -o pipefail
TAG=${1:?tag}
mkdir -p gpurun_out
OUT=gpurun_out/k4m1x2_ab_$TAG.txt
: > "$OUT"
timeout -k 10 400 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
for i in 1 2; do
  for x in 0 1; do
    echo "== RSAMD_K4M1X2=$x granule" >> "$OUT"
    RSAMD_K4M1X2=$x timeout -k 10 200 python3 tools/granule_decode_probe.py 1 64 "table:-1:-1" 2>/dev/null | grep -v amdgpu.ids >> "$OUT" || exit 1
    echo "== RSAMD_K4M1X2=$x packed" >> "$OUT"
    RSAMD_K4M1X2=$x timeout -k 10 200 python3 tools/lib_ab_same.py java-reed-solomon-distributed-file-system_amd/lib/librsamd.so --reps 1 2>/dev/null | grep -E "dec0|enc\"" | grep -v amdgpu.ids >> "$OUT" || exit 1
  done
done
cat "$OUT"
