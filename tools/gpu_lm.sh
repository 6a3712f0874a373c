#!/bin/bash
# LM refinement: the primitive / classification parity tests, classification timing, and the per-phase
# cycle profile of k_elm (dbglib/elmprof: the same sources built with -DPITT_ELM_PROF).
set -o pipefail
TAG=${1:-lm}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sphere.py tests/test_cylinder.py tests/test_cone.py tests/test_classify_gpu.py \
    tests/test_services_gpu.py tests/test_pcl_lm.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 120 python3 tools/classify_run.py 10 || exit 1
PITT_LIB_PATH=$PWD/dbglib/elmprof/libpitt_seg.so timeout -k 10 120 python tools/classify_run.py 1 > gpurun_out/${TAG}_elmprof.log 2>&1 || exit 1
grep -c PITT_ELM_PROF gpurun_out/${TAG}_elmprof.log
