#!/bin/bash
# Baseline GPU round: parity tests, then a default bench line.  Each GPU step has its own limit and
# the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
