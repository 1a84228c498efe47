# Direct file decode row mapping A/B, then the full GPU suite and the bench.
set -o pipefail
tag=${1:-r3s2m}
bash tools/gpu_direct_file.sh $tag 128 0,1 || exit 1
bash tools/gpu_quick.sh $tag || exit 1
