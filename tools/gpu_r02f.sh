#!/bin/bash
# GPU tests, the preprocess/primitive-services bench and its rocprofv3 kernel stats; each step time-limited,
# the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/bench_preprocess.py > gpurun_out/preprocess.json 2> gpurun_out/preprocess.err || exit $?
bash tools/gpu_prof_preprocess.sh r02f || exit $?
exit 0
