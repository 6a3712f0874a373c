#!/bin/bash
# The driver's command (--steps 20 --warmup 5) on the in-tree library and on abv/libpitt_seg_<name>.so,
# alternating.
set -o pipefail
V=$1; VL=$PWD/abv/libpitt_seg_$V.so
mkdir -p gpurun_out
for r in 1 2 3; do
  for lib in cur $V; do
    if [ $lib = $V ]; then export PITT_LIB_PATH=$VL; else unset PITT_LIB_PATH; fi
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/abv20_${lib}_$r.json 2> gpurun_out/abv20_${lib}_$r.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/abv20_${lib}_$r.json')); print('$lib', d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels']['k_score.first']['avg_launch_us'])"
  done
done
