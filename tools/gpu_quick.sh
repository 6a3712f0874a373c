#!/bin/bash
# Quick GPU check: plane parity tests + bench at pipeline 1 and 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_plane_gpu.py tests/test_golden.py -m gpu -q --timeout 600 -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_quick.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --pipeline 1 --no-cpu-baseline > gpurun_out/bench_p1.json 2> gpurun_out/bench_p1.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --pipeline 2 --no-cpu-baseline > gpurun_out/bench_p2.json 2> gpurun_out/bench_p2.err || exit $?
exit $rc
