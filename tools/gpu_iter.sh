#!/bin/bash
# One development iteration on the GPU box: full GPU tests, the default bench, and a kernel trace
# of a one-batch-in-flight bench (per-launch durations for tools/exp_report.py-style analysis).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-it}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/${TAG}_pytest.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_p1" -o t -f csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --pipeline 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_p1.log" 2>&1 || exit $?
exit $rc
