#!/bin/bash
# Headline repeatability: three default-length headline passes and the steady-state loop.
set -o pipefail
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline > gpurun_out/hl_$r.json 2> gpurun_out/hl_$r.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/hl_$r.json')); print('run $r', d['value'], d['ms_per_step'])"
done
timeout -k 10 200 python tools/host_enqueue.py 200 4 || exit 1
