#!/bin/bash
# Exact-walk producer change: the walk / plane / support parity tests, then config-2 timing.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_xsum_gpu.py tests/test_plane_gpu.py tests/test_golden.py tests/test_independent.py \
    tests/test_supports_clusters_gpu.py tests/test_schedule_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/xr_tests.log 2>&1 || { tail -30 gpurun_out/xr_tests.log; exit 1; }
tail -1 gpurun_out/xr_tests.log
for r in 1 2; do timeout -k 10 120 python tools/config2_run.py 40 || exit 1; done
