#!/bin/bash
# A/B of page-locking pageable caller buffers per call (host.cpp
# HostRegistration): GPU tests, then bench.py's host-inclusive legs with
# RSAMD_HOST_REGISTER=0 (pinned mirrors + host memcpy) and the default, twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
timeout -k 10 500 python3 -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread 2>&1 | tail -1 || exit 1
for r in 1 2; do
  for f in 0 1; do
    line=$(RSAMD_HOST_REGISTER=$f timeout -k 10 300 python3 bench.py --cpu-seconds 0.2 2>/dev/null) || { echo FAILED; exit 1; }
    python3 -c "import json,sys; e=json.loads(sys.argv[1])['extra']; print('round $r HOST_REGISTER=$f', ' '.join(f'{k[15:]}={v}' for k,v in e.items() if k.startswith('host_inclusive') and 'note' not in k))" "$line"
  done
done
