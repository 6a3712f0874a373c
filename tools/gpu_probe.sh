#!/bin/bash
# Probe run: op-rate microbenchmark, the independent-pin GPU tests, SQ counters of k_score.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 60 ./tools/microbench/op_rates > gpurun_out/op_rates.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_independent.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/independent_gpu.log 2>&1 || exit $?
bash tools/gpu_sq.sh ${1:-base} k_score --no-extras
