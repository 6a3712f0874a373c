#!/bin/bash
# Config 2: the single-cloud path's staging modes / chunk sizes (alternating), then the plane tests.
set -o pipefail
for r in 1 2; do
  for cfg in "0 65536" "0 131072" "1 0" "0 32768"; do
    set -- $cfg
    echo "mode $1 chunk $2: $(PITT_SINGLE_MODE=$1 PITT_SINGLE_CHUNK=$2 timeout -k 10 120 python tools/config2_run.py 40)" || exit 1
  done
done
PITT_HOST_TIMING=1 timeout -k 10 120 python tools/config2_run.py 4 2>&1 | grep pitt_plane_segment | tail -2
timeout -k 10 300 python -u -m pytest tests/test_plane_gpu.py tests/test_golden.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/c2b_tests.log 2>&1 || { tail -30 gpurun_out/c2b_tests.log; exit 1; }
tail -1 gpurun_out/c2b_tests.log
