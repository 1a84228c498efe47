# Host-API direct path: per-call page-locking cost (tools/reg_cost.py) and a
# kernel trace of pageable vs pinned encodeParity calls (tools/host_calls.py).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r3s2d}
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/hc_$tag -o run -- python3 tools/host_calls.py --calls 4 > gpurun_out/host_calls_$tag.txt 2>&1 || { tail -20 gpurun_out/host_calls_$tag.txt; exit 1; }
grep '^{' gpurun_out/host_calls_$tag.txt | cut -c1-200
for f in $(find gpurun_out/hc_$tag -name '*stats.csv'); do echo "== $f"; cut -d, -f1-4 $f | head -12; done
