#!/bin/bash
# Cone / cylinder / service-handler GPU tests only (one process, its own time limit).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cone.py tests/test_cylinder.py tests/test_services_gpu.py -m gpu -x -v \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_cone.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_cone.log
exit $rc
