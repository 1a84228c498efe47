#!/bin/bash
set -o pipefail
tag=${1:-r3e}
out=gpurun_out
mkdir -p $out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python tools/host_bisect.py > $out/host_bisect_$tag.txt 2>&1; rc=$?
grep '^{' $out/host_bisect_$tag.txt
exit $rc
