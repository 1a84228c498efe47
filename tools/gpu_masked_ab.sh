set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_granule.py tests/test_gpu_recovery.py tests/test_gpu_graphs.py tests/test_gpu_limits.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_r2bd.log 2>&1 || { tail -30 gpurun_out/pytest_r2bd.log; exit 1; }
tail -1 gpurun_out/pytest_r2bd.log
timeout -k 10 400 python3 tools/masked_ab.py tools/bin/librsamd_base.so tools/bin/librsamd_tmpl.so --reps 4 > gpurun_out/masked_ab_r2bd.txt 2>&1 || { tail -20 gpurun_out/masked_ab_r2bd.txt; exit 1; }
cat gpurun_out/masked_ab_r2bd.txt
