#!/bin/bash
# k_xrefine: its parity tests, then its counters ($PITT_REFINE_DEBUG: cycles, add-list entries per
# stream) at pipeline 1, then the default bench.  Each GPU step has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-xrdbg}
timeout -k 10 300 python -u -m pytest tests/test_xrefine_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "$OUT/${TAG}_pytest.log" 2>&1 || exit $?
PITT_REFINE_DEBUG=1 timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --pipeline 1 --no-extras --no-cpu-baseline \
    > "$OUT/${TAG}.json" 2> "$OUT/${TAG}.err" || exit $?
timeout -k 10 300 python3 bench.py --steps 40 --no-extras --no-cpu-baseline > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err" || exit $?
