#!/bin/bash
# k_score point prefetch depth A/B (abtmp/libpitt_seg_d3.so = -DPITT_SCORE_DEPTH=3), alternating, then the
# variant's plane parity tests.
set -o pipefail
for r in 1 2 3; do
  for lib in cur d3; do
    if [ $lib = d3 ]; then export PITT_LIB_PATH=$PWD/abtmp/libpitt_seg_d3.so; else unset PITT_LIB_PATH; fi
    timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline > gpurun_out/d3_${lib}_$r.json 2> gpurun_out/d3_${lib}_$r.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/d3_${lib}_$r.json')); print('$lib', d['value'], d['roofline']['frac'], d['kernels']['k_score.first']['avg_launch_us'])"
  done
done
PITT_LIB_PATH=$PWD/abtmp/libpitt_seg_d3.so timeout -k 10 300 python -u -m pytest tests/test_plane_gpu.py tests/test_golden.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/d3_tests.log 2>&1 || { tail -20 gpurun_out/d3_tests.log; exit 1; }
tail -1 gpurun_out/d3_tests.log
