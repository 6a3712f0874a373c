#!/bin/bash
# VoxelGrid per-frame timing A/B over libraries: bash tools/gpu_vox_ab.sh NAME... (cur = in-tree,
# else abv/libpitt_seg_NAME.so); two alternating rounds, each step under its own time limit.
export PYTHONPATH=$PWD
mkdir -p gpurun_out
for r in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = cur ]; then unset PITT_LIB_PATH; else export PITT_LIB_PATH=$PWD/abv/libpitt_seg_$lib.so; fi
    timeout -k 10 120 python -u tools/voxel_run.py --reps 2 > gpurun_out/voxab_${lib}_$r.log 2>&1 || { tail -20 gpurun_out/voxab_${lib}_$r.log; exit 1; }
    echo "$lib $(tail -1 gpurun_out/voxab_${lib}_$r.log)"
  done
done
