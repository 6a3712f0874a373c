#!/bin/bash
# Pipeline depth x hardware queues sweep of bench.py (batches in flight), plus a kernel + HIP API trace
# of config 5.  Each run has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-pipe}
for cfg in "3 4" "4 4" "4 8" "5 8" "6 8"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --steps 40 --no-extras --no-cpu-baseline --pipeline $1 --hw-queues $2 \
      > "$OUT/${TAG}_p$1_q$2.json" 2> "$OUT/${TAG}_p$1_q$2.err" || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d "$OUT/${TAG}_c5" -o c5 -f csv -- \
    python3 "$GRAFT_REPO_ROOT/tools/config5_run.py" 3 > "$OUT/${TAG}_c5.log" 2>&1 || exit $?
