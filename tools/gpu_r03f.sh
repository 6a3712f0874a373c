#!/bin/bash
# Round-3 final record: the -m gpu suite, smoke, the default bench line, then tools/gpu_profile.sh's
# rocprofv3 passes (kernel trace + stats of the bench, FETCH_SIZE and WRITE_SIZE passes on k_score,
# each its own run).  Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
TAG=${1:-r03f}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    > "$OUT/${TAG}_pytest_gpu.log" 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1 || exit $?
timeout -k 10 400 python bench.py > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err" || exit $?
bash tools/gpu_profile.sh "$TAG" 10 || exit $?
