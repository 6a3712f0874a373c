#!/bin/bash
# The default bench line twice (the driver's command), one step with its own time limit each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-bo}
for rep in 1 2; do
  timeout -k 10 400 python bench.py > "$OUT/${TAG}_$rep.json" 2> "$OUT/${TAG}_$rep.err" || exit $?
done
