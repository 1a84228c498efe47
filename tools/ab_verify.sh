# Verify A/B: GPU tests on the current build, then tools/verify_probe.py on an older
# build (tools/bin/old/librsamd.so, built by hand from an earlier kernels.hip) and on the current one.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_verifypin.log 2>&1 || { tail -30 gpurun_out/pytest_verifypin.log; exit 1; }
tail -1 gpurun_out/pytest_verifypin.log
for rep in 1 2; do
  echo old; RSAMD_LIB_OVERRIDE=$PWD/tools/bin/old/librsamd.so timeout -k 10 120 python3 tools/verify_probe.py 2>/dev/null || exit 1
  echo new; timeout -k 10 120 python3 tools/verify_probe.py 2>/dev/null || exit 1
done | tee gpurun_out/verify_ab.txt
