#!/bin/bash
# k_refine iteration: every plane/support parity test, then a short bench (kernel table incl. k_refine).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-refine}
timeout -k 10 600 python -u -m pytest tests/test_plane_gpu.py tests/test_shortcuts_gpu.py tests/test_golden.py \
    tests/test_supports_clusters_gpu.py tests/test_independent.py tests/test_services_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_bench.json \
    2> gpurun_out/${TAG}_bench.err || exit $?
