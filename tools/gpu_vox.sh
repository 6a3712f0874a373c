#!/bin/bash
# VoxelGrid (PCL order) A/B: the watchdog build on small sorts (if built), the voxel tests, then per-frame
# timings of abv/libpitt_seg_base.so (if present) against the in-tree library, and a rocprofv3 kernel
# trace of the in-tree one.
#   bash tools/gpu_vox.sh
export PYTHONPATH=$PWD
mkdir -p gpurun_out
if [ -f abv/libpitt_seg_isdbg.so ]; then
  PITT_LIB_PATH=$PWD/abv/libpitt_seg_isdbg.so timeout -k 10 120 python -u tools/is_debug.py > gpurun_out/isdbg.log 2>&1 || { tail -20 gpurun_out/isdbg.log; exit 1; }
  grep -c ok gpurun_out/isdbg.log; grep -i "watchdog\|MISMATCH" gpurun_out/isdbg.log && exit 1
fi
timeout -k 10 600 python -u -m pytest tests/test_voxel.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/vox_tests.log 2>&1 || { tail -30 gpurun_out/vox_tests.log; exit 1; }
tail -1 gpurun_out/vox_tests.log
if [ -f abv/libpitt_seg_base.so ]; then
  PITT_LIB_PATH=$PWD/abv/libpitt_seg_base.so timeout -k 10 300 python -u tools/voxel_run.py --reps 3 > gpurun_out/vox_base.log 2>&1 || { tail -20 gpurun_out/vox_base.log; exit 1; }
  tail -1 gpurun_out/vox_base.log
fi
timeout -k 10 300 python -u tools/voxel_run.py --reps 3 --check > gpurun_out/vox_new.log 2>&1 || { tail -20 gpurun_out/vox_new.log; exit 1; }
tail -1 gpurun_out/vox_new.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/vox_prof_new -o vox -- python3 $GRAFT_REPO_ROOT/tools/voxel_run.py --reps 2 > $GRAFT_REPO_ROOT/gpurun_out/vox_prof_new.log 2>&1
