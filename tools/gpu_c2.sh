#!/bin/bash
# Config-2 host path: single-cloud ABI timings per staging chunk size, the host phases, the single-cloud
# tests; then the default bench with the adaptive chunk schedule off (streaming continuations A/B).
set -o pipefail
TAG=${1:-r05c2}
mkdir -p gpurun_out
for c in 65536 0 131072 32768 16384; do
    echo "chunk $c: $(PITT_SINGLE_CHUNK=$c timeout -k 10 120 python tools/config2_run.py 40)" || exit 1
done
PITT_HOST_TIMING=1 timeout -k 10 120 python tools/config2_run.py 8 > gpurun_out/${TAG}_timing.log 2>&1 || exit 1
grep -c pitt_plane_segment gpurun_out/${TAG}_timing.log; tail -4 gpurun_out/${TAG}_timing.log
timeout -k 10 300 python -u -m pytest tests/test_plane_gpu.py tests/test_golden.py tests/test_schedule_gpu.py tests/test_graphs_gpu.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
echo done
