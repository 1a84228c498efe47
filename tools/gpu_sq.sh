#!/bin/bash
# SQ counter passes (instruction mix, wave-cycle breakdown, clock) on the
# measured kernel shapes: one process per workload (tools/pmc_workloads.py),
# two counter sets in separate runs (counters only: no sys/runtime trace), then
# tools/sq_summary.py into gpurun_out/sq_<tag>.json.
# Usage (via gpurun): bash tools/gpu_sq.sh [tag]
set -o pipefail
TAG=${1:-r2}${RSAMD_XORNET:+_xn$RSAMD_XORNET}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
PASS_A="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
PASS_B="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM"
PASS_C="TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_STALL TCC_BUSY GRBM_GUI_ACTIVE"
DIRS=""
for W in ${WORKLOADS:-enc42 enc104 dec104 enc104p maskbits104}; do
  for P in ${PASSES:-A B}; do
    case $P in A) C=$PASS_A ;; B) C=$PASS_B ;; C) C=$PASS_C ;; esac
    echo "== $W pass $P $(date +%T)"
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$OUT/sq_${TAG}_${W}_$P" -o run -- \
        python3 "$R/tools/pmc_workloads.py" $W > "$OUT/sq_${TAG}_${W}_$P.log" 2>&1 || { tail -20 "$OUT/sq_${TAG}_${W}_$P.log"; exit 1; }
    DIRS="$DIRS $W:$OUT/sq_${TAG}_${W}_$P"
  done
done
python3 tools/sq_summary.py "$OUT/sq_${TAG}.json" $DIRS
echo "== done $(date +%T)"
