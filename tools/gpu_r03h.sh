#!/bin/bash
# Round-3 re-entry check: the -m gpu suite and smoke on the rebuilt library, then the pipeline depth x
# hardware queue sweep at the driver's 20 steps.  Each GPU step has its own time limit; the chain
# stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; TAG=${1:-r03h}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    > "$OUT/${TAG}_pytest_gpu.log" 2>&1 || exit $?
tail -1 "$OUT/${TAG}_pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1 || exit $?
bash tools/gpu_pipe_sweep.sh "$TAG" 20 "4 8" "5 8" "5 16" "6 16" "4 8" "5 16" "6 16"
