# Tiled direct file decode: its tests and the A/B against the untiled form,
# then the full GPU suite and the bench.
set -o pipefail
tag=${1:-r3s2p}
bash tools/gpu_direct_file.sh $tag 128 0,1 || exit 1
bash tools/gpu_quick.sh $tag || exit 1
