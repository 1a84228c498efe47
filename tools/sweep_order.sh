#!/bin/bash
# Block-order sweep on the real encode kernel across shard sizes
# (tools/ab_order_encode.sh per size).  Usage (via gpurun): bash tools/sweep_order.sh
set -o pipefail
C=${CONFIGS:-ROT=0,XCD=0 ROT=0,XCD=1 ROT=127,XCD=0 ROT=383,XCD=0 ROT=129,XCD=0 ROT=385,XCD=0}
SIZES=${SIZES:-262144:16384 524288:8192 1048576:4096 2097152:2048 4194304:1024 8388608:512}
for a in $SIZES; do
  CONFIGS="$C" bash tools/ab_order_encode.sh 1 --shard-bytes ${a%%:*} --stripes ${a##*:} ${EXTRA:-} || exit 1
done
