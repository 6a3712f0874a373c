#!/bin/bash
# Headline with the batch refinement through the exact walk (PITT_XS_MAX_FRAMES large) against the
# per-frame chain, at the driver's 20 steps and at 200.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for xs in 8 100000; do
    for k in 20 200; do
      PITT_XS_MAX_FRAMES=$xs timeout -k 10 200 python bench.py --steps $k --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/xs_${xs}_${k}_$r.json 2> gpurun_out/xs_${xs}_${k}_$r.err || exit 1
      python -c "import json; d=json.load(open('gpurun_out/xs_${xs}_${k}_$r.json')); print('xs=$xs k=$k', d['value'], d['ms_per_step'], {n: v['us_per_batch'] for n, v in d['kernels'].items()})"
    done
  done
done
