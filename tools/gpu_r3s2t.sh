# Runtime-k masked kernel (per-stripe patterns, other codes): group size
# (gen1 = one input ahead, tuning = groups of 4) x occupancy cap, builds
# alternated; then the GPU tests that use it.
# Builds (in csrc/): make TUNING=1 OUT=../../build/ab/tuning OBJ=../../build/ab/tuning/obj, and the same
# with OUT/OBJ under build/ab/gen1 and KDEFS=-DRSAMD_GEN_GROUP=1.
set -o pipefail
tag=${1:-r3s2t}
mkdir -p gpurun_out
out=gpurun_out/masked_gen_$tag.txt
for rep in 1 2; do
  for lib in gen1 tuning; do
    echo "# lib $lib rep $rep" >> $out
    timeout -k 10 200 python3 tools/occ_sweep2.py --family masked --lib build/ab/$lib/librsamd.so --reps 1 \
      --shapes 6p3_granule_3random,8p4_granule_2random,17p3_granule_3random --pads 0,10240,12544 >> $out 2>&1 || { tail $out; exit 1; }
  done
done
grep -v amdgpu.ids $out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_random.py tests/test_gpu_parity.py tests/test_gpu_recovery.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_masked_$tag.log 2>&1 || { tail -30 gpurun_out/pytest_masked_$tag.log; exit 1; }
tail -1 gpurun_out/pytest_masked_$tag.log
