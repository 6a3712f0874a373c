export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r06g_bench.json 2> gpurun_out/r06g_bench.log || { tail -20 gpurun_out/r06g_bench.log; exit 1; }
timeout -k 10 200 python -u tools/voxel_run.py --reps 3 --check > gpurun_out/r06g_voxel.log 2>&1 || { tail -20 gpurun_out/r06g_voxel.log; exit 1; }
tail -1 gpurun_out/r06g_voxel.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06g_voxprof -o vox -- python3 $GRAFT_REPO_ROOT/tools/voxel_run.py --reps 2 > $GRAFT_REPO_ROOT/gpurun_out/r06g_voxprof.log 2>&1
