#!/bin/bash
# VoxelGrid timing of exp_libs/<variant>/libpitt_seg.so builds against the in-tree library.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python tools/bench_preprocess.py --frames 16 --reps 3 > gpurun_out/vsw_base.json 2> gpurun_out/vsw_base.err || exit $?
for v in "$@"; do
    PITT_LIB_PATH=$PWD/exp_libs/$v/libpitt_seg.so timeout -k 10 120 python tools/bench_preprocess.py --frames 16 --reps 3 \
        > gpurun_out/vsw_$v.json 2> gpurun_out/vsw_$v.err || exit $?
done
