#!/bin/bash
# A/B of the host pipeline's stream layout and chunk count (host.cpp
# run_chunks): bench.py's host-inclusive legs under each setting, twice.
# Usage (via gpurun):  bash tools/ab_pipe.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
SETTINGS=${SETTINGS:-"RSAMD_PIPE_STREAMS=2 RSAMD_PIPE_STREAMS=3 RSAMD_CHUNKS=12 RSAMD_CHUNKS=16"}
for r in $(seq 1 ${ROUNDS:-2}); do
  for s in $SETTINGS; do
    line=$(env "$s" timeout -k 10 120 python3 tools/host_legs.py 2>/dev/null) || { echo "FAILED $s"; exit 1; }
    echo "round $r $s $line"
  done
done
