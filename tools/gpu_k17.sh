# Compiled 17+m shapes (the upstream library's benchmark code) against the
# runtime-k kernel: occupancy sweep, builds alternated.
# Builds (in csrc/): build/ab/before = TUNING build without the K = 17 cases,
# build/ab/tuning = TUNING build with them.
set -o pipefail
tag=${1:-k17}
mkdir -p gpurun_out
out=gpurun_out/k17_$tag.txt
for rep in 1 2; do
  for lib in before tuning; do
    echo "# lib $lib rep $rep" >> $out
    timeout -k 10 200 python3 tools/occ_sweep.py --lib build/ab/$lib/librsamd.so --reps 1 \
      --shapes 17p3g_enc,17p3g_dec012 --pads 0,8192,10240,12544,16384 >> $out 2>&1 || { tail $out; exit 1; }
  done
done
grep -v amdgpu.ids $out
