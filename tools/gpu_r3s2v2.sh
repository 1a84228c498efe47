# Product build with the compiled 6+m, 8+m and 17+m shapes: their rates, the full GPU
# suite, smoke and the bench.
set -o pipefail
tag=${1:-r3s2v2}
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/occ_sweep.py --lib java-reed-solomon-distributed-file-system_amd/lib/librsamd.so --reps 2 \
  --shapes 17p3g_enc,17p3g_dec012,8p4g_enc,8p4g_dec0,6p3g_enc,6p3g_dec01 --pads 0 > gpurun_out/k17_product_$tag.txt 2>&1 || { tail gpurun_out/k17_product_$tag.txt; exit 1; }
grep "^{" gpurun_out/k17_product_$tag.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { cat gpurun_out/smoke_$tag.log; exit 1; }
tail -1 gpurun_out/smoke_$tag.log
bash tools/gpu_quick.sh $tag || exit 1
