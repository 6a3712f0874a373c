#!/bin/bash
# Round-3 check after the classification work: -m gpu suite, smoke, default bench, and a kernel-trace
# --stats profile of the bench.  Each GPU step has its own time limit; the chain stops at a failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
TAG=${1:-r03b}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    > "$OUT/${TAG}_pytest_gpu.log" 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1 || exit $?
timeout -k 10 400 python bench.py > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o bench -f csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$OUT/${TAG}_prof.log" 2>&1 || exit $?
