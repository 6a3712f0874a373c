#!/bin/bash
# The primitive services' refinement (PCL's float LM on the device, csrc/elm.hpp) against the oracle.
set -o pipefail
TAG=${1:-r04lm}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_sphere.py tests/test_cylinder.py tests/test_cone.py \
    tests/test_services_gpu.py tests/test_classify_gpu.py -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/${TAG}_pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/${TAG}_pytest.log | tail -60
exit $rc
