#!/bin/bash
# SQ issue/stall counters for one kernel (default k_score) over a short bench.py run.
#   bash tools/gpu_sq.sh <tag> [kernel-regex] [extra bench args...]
# Output: gpurun_out/sq_<tag>_{a,b}/ (two PMC passes, 8 SQ slots each).
set -o pipefail
ROOTDIR="$GRAFT_REPO_ROOT"
TAG=${1:-sq}
KRE=${2:-k_score}
shift 2
cd /tmp && export TMPDIR=/tmp
OUT="$ROOTDIR/gpurun_out"
mkdir -p "$OUT"
BENCH="$ROOTDIR/bench.py --steps 2 --warmup 1 --pipeline 1 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS --kernel-include-regex "$KRE" \
    -d "$OUT/sq_${TAG}_a" -o a -f csv -- python3 $BENCH > "$OUT/sq_${TAG}_a.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE \
    SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU --kernel-include-regex "$KRE" \
    -d "$OUT/sq_${TAG}_b" -o b -f csv -- python3 $BENCH > "$OUT/sq_${TAG}_b.log" 2>&1 || exit $?
echo done > "$OUT/sq_${TAG}_done"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH \
    SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --kernel-include-regex "$KRE" \
    -d "$OUT/sq_${TAG}_c" -o c -f csv -- python3 $BENCH > "$OUT/sq_${TAG}_c.log" 2>&1 || exit $?
echo done > "$OUT/sq_${TAG}_done"
