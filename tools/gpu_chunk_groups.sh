#!/bin/bash
# Row f2 at S = 1000 (the master's chunk groups): recovery and 8-byte-kernel
# GPU tests, then tools/chunk_group_probe.py with the in-tree build, an A/B
# build (optional $2: a variant librsamd.so), and without the 8-byte-aligned
# kernels (RSAMD_MASKED8=0: the byte kernel).
# Usage (via gpurun): bash tools/gpu_chunk_groups.sh TAG [variant.so]
set -o pipefail
TAG=${1:?tag}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests \
    -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_recovery_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_recovery_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_recovery_$TAG.log
timeout -k 10 300 python3 tools/chunk_group_probe.py --reps 2 > gpurun_out/chunk_groups_$TAG.txt 2>&1 || { tail -20 gpurun_out/chunk_groups_$TAG.txt; exit 1; }
if [ -n "$2" ]; then
  timeout -k 10 300 python3 tools/chunk_group_probe.py --reps 2 --strides 1000 --lib "$2" >> gpurun_out/chunk_groups_$TAG.txt 2>&1 || { tail -20 gpurun_out/chunk_groups_$TAG.txt; exit 1; }
fi
RSAMD_MASKED8=0 timeout -k 10 300 python3 tools/chunk_group_probe.py --reps 1 --strides 1000 \
    >> gpurun_out/chunk_groups_$TAG.txt 2>&1 || { tail -20 gpurun_out/chunk_groups_$TAG.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/chunk_groups_$TAG.txt
