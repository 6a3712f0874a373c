#!/bin/bash
set -o pipefail
ROOTDIR="$GRAFT_REPO_ROOT"; TAG=${1:-t}; shift
cd /tmp && export TMPDIR=/tmp
OUT="$ROOTDIR/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace -d "$OUT/prof_${TAG}" -o trace -f csv -- python3 "$ROOTDIR/bench.py" "$@" \
    > "$OUT/prof_${TAG}.log" 2>&1
