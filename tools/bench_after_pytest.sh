#!/bin/bash
# Does the headline encode depend on what ran on the GPU before it?  bench.py
# (--no-extras) fresh, then after the GPU test suite, then after each of the
# heavier GPU test files alone.  Usage (via gpurun): bash tools/bench_after_pytest.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
frac() { timeout -k 10 120 python3 bench.py --no-extras --steps 30 | python3 -c "import json,sys; d=json.load(sys.stdin)['roofline']; print('$1', d['frac'], d['avg_launch_ms'])"; }
frac fresh && frac fresh || exit 1
timeout -k 10 500 python3 -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread 2>&1 | tail -1
frac "after full pytest" && frac "after full pytest" && frac "after full pytest" || exit 1
for t in ${TESTS:-tests/test_gpu_limits.py tests/test_gpu_reference_test.py tests/test_gpu_parity.py}; do
  timeout -k 10 300 python3 -m pytest $t -x -q -m gpu --timeout 200 --timeout-method thread 2>&1 | tail -1
  frac "after $t" || exit 1
done
