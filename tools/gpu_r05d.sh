#!/bin/bash
# Round-5: the graph tests, then the kernel traces (config 5, classification, config 2).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_graphs_gpu.py -m gpu -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r05d_graphs.log 2>&1
rc=$?; tail -3 gpurun_out/r05d_graphs.log
if grep -qiE "illegal memory access|memory access fault|HSA_STATUS_ERROR" gpurun_out/r05d_graphs.log; then exit 3; fi
[ $rc -le 1 ] || exit $rc
bash tools/gpu_prof_r05.sh r05d
