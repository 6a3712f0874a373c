#!/bin/bash
# LM change check: primitive / classification parity tests, classification timing, the cone job's profile.
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_sphere.py tests/test_cylinder.py tests/test_cone.py tests/test_classify_gpu.py \
    tests/test_services_gpu.py tests/test_pcl_lm.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/lm2_tests.log 2>&1 || { tail -30 gpurun_out/lm2_tests.log; exit 1; }
tail -1 gpurun_out/lm2_tests.log
for r in 1 2; do timeout -k 10 120 python3 tools/classify_run.py 20 | cut -c1-24 || exit 1; done
bash tools/gpu_lmprof.sh
