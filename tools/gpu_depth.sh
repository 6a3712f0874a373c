#!/bin/bash
# Pipeline depth at the driver's 20 steps and at 200, alternating on one box.
set -o pipefail
for r in 1 2; do
  for p in 3 4 5; do
    for k in 20 200; do
      timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --steps $k --warmup 5 --pipeline $p > gpurun_out/dp_${p}_${k}_$r.json 2> /dev/null || exit 1
      python -c "import json; d=json.load(open('gpurun_out/dp_${p}_${k}_$r.json')); print('depth $p steps $k', d['value'], d['ms_per_step'])"
    done
  done
done
