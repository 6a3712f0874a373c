#!/bin/bash
# First scoring chunk size A/B (PITT_FIRST_CHUNK builds in abtmp/), 200 steps, alternating on one box.
set -o pipefail
for r in 1 2; do
  for v in 32 24 28 40; do
    if [ $v = 32 ]; then unset PITT_LIB_PATH; else export PITT_LIB_PATH=$PWD/abtmp/libpitt_seg_fc$v.so; fi
    timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline > gpurun_out/fc_${v}_$r.json 2> /dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/fc_${v}_$r.json')); k=d['kernels']; print('first $v', d['value'], d['roofline']['frac'], k['k_score']['us_per_batch'], k['k_score.first']['avg_launch_us'])"
  done
done
