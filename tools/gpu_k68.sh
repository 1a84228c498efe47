# Compiled 6+m / 8+m shapes (A/B build, KDEFS=-DRSAMD_TRY_K68=1, build/ab/k68)
# against the runtime-k kernel (build/ab/before): occupancy sweep, alternated.
set -o pipefail
tag=${1:-k68}
mkdir -p gpurun_out
out=gpurun_out/k68_$tag.txt
for rep in 1 2; do
  for lib in before k68; do
    echo "# lib $lib rep $rep" >> $out
    timeout -k 10 200 python3 tools/occ_sweep.py --lib build/ab/$lib/librsamd.so --reps 1 \
      --shapes 8p4g_enc,8p4g_dec0,6p3g_enc,6p3g_dec01 --pads 0,8192,10240,12544,14848,16384 >> $out 2>&1 || { tail $out; exit 1; }
  done
done
grep -v amdgpu.ids $out
