#!/bin/bash
# Round-5 kernel traces: config 5 (device path only), the ten-cluster classification, config 2.
set -o pipefail
ROOTDIR="$GRAFT_REPO_ROOT"
TAG=${1:-r05}
cd /tmp && export TMPDIR=/tmp
OUT="$ROOTDIR/gpurun_out"
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_c5" -o trace -f csv -- \
    python3 "$ROOTDIR/tools/config5_run.py" 3 --dev-only > "$OUT/${TAG}_c5.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_cls" -o trace -f csv -- \
    python3 "$ROOTDIR/tools/classify_run.py" 3 > "$OUT/${TAG}_cls.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_c2" -o trace -f csv -- \
    python3 "$ROOTDIR/tools/config2_run.py" 5 > "$OUT/${TAG}_c2.log" 2>&1 || exit $?
tail -1 "$OUT/${TAG}_c5.log"; tail -1 "$OUT/${TAG}_cls.log"; tail -1 "$OUT/${TAG}_c2.log"
