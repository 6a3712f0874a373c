#!/bin/bash
# Headline A/B: the current library against an earlier build (abtmp/libpitt_seg_r05f.so), alternating.
set -o pipefail
for r in 1 2 3; do
  for lib in cur old; do
    if [ $lib = old ]; then export PITT_LIB_PATH=$PWD/abtmp/libpitt_seg_r05f.so; else unset PITT_LIB_PATH; fi
    timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline > gpurun_out/hlab_${lib}_$r.json 2> gpurun_out/hlab_${lib}_$r.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/hlab_${lib}_$r.json')); print('$lib run $r', d['value'], d['ms_per_step'], d['library_sha16'])"
  done
done
