#!/bin/bash
# k_score iteration: plane parity tests, then a short bench (no CPU baseline).  Each GPU step has its
# own limit; the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-score}
timeout -k 10 600 python -u -m pytest tests/test_plane_gpu.py tests/test_shortcuts_gpu.py -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.json \
    2> gpurun_out/${TAG}_bench.err || exit $?
