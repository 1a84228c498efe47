# Host file API direct path: GPU tests of the direct paths, per-call rates by
# buffer kind and block count, and a kernel trace of the same calls.
set -o pipefail
tag=${1:-dfile}
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_direct.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_direct_$tag.log 2>&1 || { tail -30 gpurun_out/pytest_direct_$tag.log; exit 1; }
tail -1 gpurun_out/pytest_direct_$tag.log
timeout -k 10 300 python3 tools/direct_file_probe.py --lib build/ab/tuning/librsamd.so --blocks ${2:-128,256,512} --rows ${3:-1} > gpurun_out/direct_file_$tag.txt 2>&1 || { tail gpurun_out/direct_file_$tag.txt; exit 1; }
grep "^{" gpurun_out/direct_file_$tag.txt
