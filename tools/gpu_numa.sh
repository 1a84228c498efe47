# Host legs (direct path) with the process where the scheduler put it and
# bound to the GPU's NUMA node, alternated.
set -o pipefail
tag=${1:-numa}
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python3 tools/numa_probe.py >> gpurun_out/numa_$tag.txt 2>&1 || { tail gpurun_out/numa_$tag.txt; exit 1; }
  timeout -k 10 200 python3 tools/numa_probe.py --bind >> gpurun_out/numa_$tag.txt 2>&1 || { tail gpurun_out/numa_$tag.txt; exit 1; }
done
grep "^{" gpurun_out/numa_$tag.txt | cut -c1-420
