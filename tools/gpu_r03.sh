#!/bin/bash
# Round-3 GPU call: the -m gpu suite, then a kernel trace of the 40-step bench and a kernel + HIP API
# trace of config 5.  Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
TAG=${1:-r03}
SKIP_TESTS=${SKIP_TESTS:-0}
if [ "$SKIP_TESTS" != "1" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
      > "$OUT/${TAG}_pytest_gpu.log" 2>&1 || exit $?
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/${TAG}_trace" -o trace -f csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 40 --no-extras --no-cpu-baseline > "$OUT/${TAG}_trace.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d "$OUT/${TAG}_c5" -o c5 -f csv -- \
    python3 "$GRAFT_REPO_ROOT/tools/config5_run.py" 3 > "$OUT/${TAG}_c5.log" 2>&1 || exit $?
