#!/bin/bash
# rocprofv3 kernel trace + stats over tools/bench_preprocess.py (VoxelGrid / NormalEstimation kernels).
set -o pipefail
ROOTDIR="$GRAFT_REPO_ROOT"
TAG=${1:-pre}
cd /tmp && export TMPDIR=/tmp
OUT="$ROOTDIR/gpurun_out"
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${TAG}" -o trace -f csv -- \
    python3 "$ROOTDIR/tools/bench_preprocess.py" --frames 16 --reps 2 > "$OUT/prof_${TAG}.log" 2>&1 || exit $?
