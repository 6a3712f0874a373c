#!/bin/bash
# Kernel trace of the ten-cluster classification (tools/classify_run.py), for tools/cls_timeline.py.
set -o pipefail
TAG=${1:-clst}
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}" -o trace -f csv -- \
    python3 "$R/tools/classify_run.py" 3 > "$R/gpurun_out/${TAG}.log" 2>&1 || exit $?
tail -1 "$R/gpurun_out/${TAG}.log"
