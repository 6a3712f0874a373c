#!/bin/bash
# One GPU-box round: parity tests, smoke, bench, rocprof kernel trace.  Each GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
STEP=${1:-all}
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
exit $rc
