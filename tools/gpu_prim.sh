#!/bin/bash
# Primitive services: their GPU tests, then the preprocess/primitives bench; each step time-limited.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cone.py tests/test_cylinder.py tests/test_sphere.py tests/test_services_gpu.py -m gpu -x -v \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_prim.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_prim.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/bench_preprocess.py > gpurun_out/preprocess.json 2> gpurun_out/preprocess.err || exit $?
exit 0
