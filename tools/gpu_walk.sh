#!/bin/bash
# Round-5: the exact-walk tests, then the config-2 / config-5 traces.
set -o pipefail
TAG=${1:-walk}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_xsum_gpu.py tests/test_golden.py tests/test_supports_clusters_gpu.py tests/test_independent.py tests/test_services_gpu.py -m gpu -x -v \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_c5" -o trace -f csv -- \
    python3 "$R/tools/config5_run.py" 3 --dev-only > "$R/gpurun_out/${TAG}_c5.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_c2" -o trace -f csv -- \
    python3 "$R/tools/config2_run.py" 5 > "$R/gpurun_out/${TAG}_c2.log" 2>&1 || exit $?
grep config "$R/gpurun_out/${TAG}_c5.log" "$R/gpurun_out/${TAG}_c2.log" | grep -v rocprof
python3 "$R/tools/config5_run.py" 5 --dev-only
python3 "$R/tools/config2_run.py" 10
