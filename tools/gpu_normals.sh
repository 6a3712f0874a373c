#!/bin/bash
# NormalEstimation + VoxelGrid: GPU parity tests, then the preprocessing throughput tool.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_normals.py tests/test_voxel.py -m gpu -x -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/normals_gpu.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_preprocess.py --frames 64 --reps 5 > gpurun_out/preprocess.json \
    2> gpurun_out/preprocess.err || exit $?
