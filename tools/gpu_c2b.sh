#!/bin/bash
# Config 2: the single-cloud path's staging modes (alternating), then the plane tests on the default.
set -o pipefail
for r in 1 2; do
  for m in 1 3 0 2; do
    echo "mode $m: $(PITT_SINGLE_MODE=$m timeout -k 10 120 python tools/config2_run.py 40)" || exit 1
  done
done
for m in 1 3; do PITT_HOST_TIMING=1 PITT_SINGLE_MODE=$m timeout -k 10 120 python tools/config2_run.py 4 2>&1 | grep pitt_plane_segment | tail -1; done
for m in 1 3 0; do
PITT_SINGLE_MODE=$m timeout -k 10 300 python -u -m pytest tests/test_plane_gpu.py tests/test_golden.py tests/test_schedule_gpu.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/c2b_tests_$m.log 2>&1 || { tail -30 gpurun_out/c2b_tests_$m.log; exit 1; }
echo "mode $m tests: $(tail -1 gpurun_out/c2b_tests_$m.log)"
done
