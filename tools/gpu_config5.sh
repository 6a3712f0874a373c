#!/bin/bash
# Config 5 iteration: support/cluster parity tests, then the timed config-5 run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-c5}
timeout -k 10 400 python -u -m pytest tests/test_supports_clusters_gpu.py tests/test_golden.py tests/test_independent.py \
    tests/test_services_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_pytest.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/config5_run.py 5 > gpurun_out/${TAG}_run.log 2>&1 || exit $?
