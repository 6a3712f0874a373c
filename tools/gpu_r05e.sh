#!/bin/bash
# Round-5 pass: the exact-walk tests first (fast feedback), the whole -m gpu suite, the default bench
# line, then the kernel traces (config 5, classification, config 2).  A fault or time limit stops it.
set -o pipefail
TAG=${1:-r05e}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_xsum_gpu.py tests/test_golden.py -m gpu -x -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_walk.log 2>&1 || { tail -30 gpurun_out/${TAG}_walk.log; exit 1; }
tail -1 gpurun_out/${TAG}_walk.log
bash tools/gpu_r05.sh $TAG
rc=$?
[ $rc -le 1 ] || exit $rc
bash tools/gpu_prof_r05.sh $TAG
