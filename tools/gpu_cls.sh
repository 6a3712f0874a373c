#!/bin/bash
# Round-5: the primitive-service parity tests and the classification timing / trace.
set -o pipefail
TAG=${1:-cls}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sphere.py tests/test_cylinder.py tests/test_cone.py tests/test_classify_gpu.py \
    tests/test_services_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
python3 tools/classify_run.py 10
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_cls" -o trace -f csv -- \
    python3 "$R/tools/classify_run.py" 3 > "$R/gpurun_out/${TAG}_cls.log" 2>&1 || exit $?
