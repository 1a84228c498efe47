# Product build after the masked runtime-k change: other codes' per-stripe
# rates, then the full GPU suite, smoke and the bench.
set -o pipefail
tag=${1:-r3s2u}
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/occ_sweep2.py --family masked --lib java-reed-solomon-distributed-file-system_amd/lib/librsamd.so --reps 2 \
  --shapes 6p3_granule_3random,8p4_granule_2random,17p3_granule_3random --pads 0 > gpurun_out/masked_product_$tag.txt 2>&1 || { tail gpurun_out/masked_product_$tag.txt; exit 1; }
grep "^{" gpurun_out/masked_product_$tag.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { cat gpurun_out/smoke_$tag.log; exit 1; }
tail -1 gpurun_out/smoke_$tag.log
bash tools/gpu_quick.sh $tag || exit 1
