# Runtime-k kernel in the product build (groups of 4, capped): other codes'
# rates, then the full GPU suite and the bench.
set -o pipefail
tag=${1:-r3s2r}
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/occ_sweep.py --lib java-reed-solomon-distributed-file-system_amd/lib/librsamd.so --reps 2 \
  --shapes 17p3g_enc,17p3g_dec012,8p4g_enc,8p4g_dec0,6p3g_enc,6p3g_dec01 --pads 0 > gpurun_out/gen_product_$tag.txt 2>&1 || { tail gpurun_out/gen_product_$tag.txt; exit 1; }
grep "^{" gpurun_out/gen_product_$tag.txt
bash tools/gpu_quick.sh $tag || exit 1
