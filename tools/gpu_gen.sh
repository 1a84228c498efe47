# Runtime-k kernel: input group size (RSAMD_GEN_GROUP builds) x occupancy
# cap on the codes outside the compiled shapes; builds alternated.
# Builds (in csrc/): for G in 1 2 4 8: make TUNING=1 OUT=../../build/ab/gen$G OBJ=../../build/ab/gen$G/obj KDEFS=-DRSAMD_GEN_GROUP=$G
set -o pipefail
tag=${1:-gen}
mkdir -p gpurun_out
out=gpurun_out/gen_$tag.txt
for rep in 1 2; do
  for G in 1 2 4 8; do
    echo "# lib gen$G rep $rep" >> $out
    timeout -k 10 200 python3 tools/occ_sweep.py --lib build/ab/gen$G/librsamd.so --reps 1 \
      --shapes 17p3g_enc,17p3g_dec012,8p4g_enc,8p4g_dec0,6p3g_enc,6p3g_dec01 --pads 0,8192,10240,12544,16384 >> $out 2>&1 || { tail $out; exit 1; }
  done
done
cat $out
