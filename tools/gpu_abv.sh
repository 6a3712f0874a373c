#!/bin/bash
# A/B of one variant library (abv/libpitt_seg_<name>.so, from tools/build_variant.sh) against the
# in-tree library: the variant's plane parity tests first, then 3 alternating bench runs.
#   bash tools/gpu_abv.sh <name>
set -o pipefail
V=$1; VL=$PWD/abv/libpitt_seg_$V.so
mkdir -p gpurun_out
PITT_LIB_PATH=$VL timeout -k 10 300 python -u -m pytest tests/test_plane_gpu.py tests/test_golden.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/abv_${V}_tests.log 2>&1 || { tail -20 gpurun_out/abv_${V}_tests.log; exit 1; }
tail -1 gpurun_out/abv_${V}_tests.log
for r in 1 2 3; do
  for lib in cur $V; do
    if [ $lib = $V ]; then export PITT_LIB_PATH=$VL; else unset PITT_LIB_PATH; fi
    timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline > gpurun_out/abv_${lib}_$r.json 2> gpurun_out/abv_${lib}_$r.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/abv_${lib}_$r.json')); print('$lib', d['value'], d['roofline']['frac'], d['kernels']['k_score.first']['avg_launch_us'])"
  done
done
