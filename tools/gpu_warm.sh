#!/bin/bash
# The driver's 20 timed steps after 5, 50 and 300 warm-up steps (is the 20-step gap the clocks?).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for w in 5 50 300; do
    timeout -k 10 200 python bench.py --steps 20 --warmup $w --no-extras --no-cpu-baseline > gpurun_out/warm_${w}_$r.json 2> gpurun_out/warm_${w}_$r.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/warm_${w}_$r.json')); print('$w', d['value'], d['ms_per_step'])"
  done
done
