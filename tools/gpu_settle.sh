#!/bin/bash
# The driver's 20 timed steps after 300, 1000 and 2000 untimed settle steps, alternating.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for st in 300 1000 2000; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --settle-steps $st --no-extras --no-cpu-baseline > gpurun_out/settle_${st}_$r.json 2> gpurun_out/settle_${st}_$r.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/settle_${st}_$r.json')); print('$st', d['value'], d['ms_per_step'])"
  done
done
