#!/bin/bash
# rocprofv3 kernel trace + stats of the config-5 run (find_supports + clusters on 1.2M points).
set -o pipefail
ROOTDIR="$GRAFT_REPO_ROOT"
TAG=${1:-c5}
cd /tmp && export TMPDIR=/tmp
OUT="$ROOTDIR/gpurun_out"
mkdir -p "$OUT"
timeout -k 10 300 python3 "$ROOTDIR/tools/config5_run.py" 5 > "$OUT/${TAG}_run.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_trace" -o trace -f csv -- \
    python3 "$ROOTDIR/tools/config5_run.py" 3 > "$OUT/${TAG}_trace.log" 2>&1 || exit $?
