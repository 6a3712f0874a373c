#!/bin/bash
# k_xrefine check: its parity tests, the plane parity suite and the score-path variants, then the
# default bench and an A/B against the serial chain ($PITT_XREFINE=0), then a kernel trace at
# pipeline 1.  Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-xr}
timeout -k 10 400 python -u -m pytest tests/test_xrefine_gpu.py tests/test_plane_gpu.py tests/test_shortcuts_gpu.py \
    -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/${TAG}_pytest.log" 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 40 --no-extras --no-cpu-baseline > "$OUT/${TAG}_bench1.json" 2> "$OUT/${TAG}_bench1.err" || exit $?
PITT_XREFINE=0 timeout -k 10 300 python3 bench.py --steps 40 --no-extras --no-cpu-baseline > "$OUT/${TAG}_bench0.json" 2> "$OUT/${TAG}_bench0.err" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o p -f csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --pipeline 1 --no-extras --no-cpu-baseline > "$OUT/${TAG}_prof.log" 2>&1 || exit $?
