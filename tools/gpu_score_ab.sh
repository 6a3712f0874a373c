#!/bin/bash
# k_score candidate: plane parity tests, then an A/B against exp_libs/<B>.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; B=${2:-base}; ROUNDS=${3:-2}
timeout -k 10 400 python -u -m pytest tests/test_plane_gpu.py tests/test_shortcuts_gpu.py tests/test_golden.py \
    tests/test_independent.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_pytest.log 2>&1 || exit $?
bash tools/gpu_ab.sh $TAG $B $ROUNDS
